"""Synthetic workload of BASELINE.json configs[3].

128-taxon Kingman coalescent tree (in the style of scripts/simulate.py:14,
``treesim.pure_kingman_tree``), scaled to a root height of 0.5
substitutions/site; GTR exchangeabilities (4, 40, 2, 2, 50, 1) normalised,
frequencies (0.33, 0.25, 0.16, 0.26) (scripts/simulate.py:22-24); Weibull
shape 0.5 with C = 4; 1,000,000 simulated sites, 1 % gap characters; then
pattern-compressed exactly like the real alignments (phylostan_amd.data).
Deterministic for a given seed (numpy PCG64).
"""
import numpy as np

from . import data, models
from .treeio import Node, Taxon, Tree

GTR_RATES = np.array([4.0, 40.0, 2.0, 2.0, 50.0, 1.0])
FREQS = np.array([0.33, 0.25, 0.16, 0.26])


def kingman_tree(n, rng, root_height=0.5):
    nodes = []
    taxa = []
    for i in range(n):
        nd = Node("t%d" % (i + 1))
        t = Taxon(nd.label)
        nd.taxon = t
        taxa.append(t)
        nodes.append(nd)
    height = {nd: 0.0 for nd in nodes}
    now = 0.0
    active = list(nodes)
    while len(active) > 1:
        k = len(active)
        now += rng.exponential(1.0 / (k * (k - 1) / 2.0))
        i, j = rng.choice(k, 2, replace=False)
        a, b = active[i], active[j]
        for idx in sorted((i, j), reverse=True):
            active.pop(idx)
        p = Node()
        p.add_child(a)
        p.add_child(b)
        height[p] = now
        active.append(p)
    root = active[0]
    scale = root_height / height[root]
    for nd in root.preorder_iter():
        if nd.parent_node is not None:
            nd.edge_length = (height[nd.parent_node] - height[nd]) * scale
    return Tree(root, taxa)


def simulate(n_taxa=128, n_sites=1_000_000, C=4, wshape=0.5, gap_frac=0.01, seed=0):
    """Returns (PhyloData, params) with params = dict(blens, freqs, rates, rs, ps)."""
    rng = np.random.default_rng(seed)
    tree = kingman_tree(n_taxa, rng)
    data.setup_indexes(tree)
    data.setup_dates(tree)
    S = n_taxa
    rates = GTR_RATES / GTR_RATES.sum()
    rs, ps = models.weibull_site_rates(wshape, C)
    Q, lam, V, Vinv, *_ = models.eigen_system(FREQS, rates)
    cat = rng.integers(0, C, n_sites)
    cat4 = (cat * 4).astype(np.intp)
    states = {}
    root = tree.seed_node
    states[root] = rng.choice(4, size=n_sites, p=FREQS).astype(np.uint8)
    blens = np.zeros(2 * S - 2)
    for nd in tree.preorder_node_iter():
        if nd.parent_node is None:
            continue
        blens[nd.index - 1] = nd.edge_length
        parent = states[nd.parent_node]
        u = rng.random(n_sites)
        # cumulative transition rows of every (category, parent state), then
        # per site: child = #{thresholds below u} (three table gathers)
        cum = np.empty((C, 4, 4))
        for c in range(C):
            P = (V * np.exp(lam * nd.edge_length * rs[c])[None, :]) @ Vinv
            cum[c] = np.cumsum(np.clip(P, 0.0, None), axis=1)
            cum[c] /= cum[c][:, -1:]
        flat = cum.reshape(C * 4, 4)
        idx = cat4 + parent
        child = (u > flat[:, 0][idx]).view(np.uint8).copy()
        child += (u > flat[:, 1][idx]).view(np.uint8)
        child += (u > flat[:, 2][idx]).view(np.uint8)
        states[nd] = child
    chars = np.empty((S, n_sites), dtype=np.uint8)
    lut = np.frombuffer(b"ACGT", dtype=np.uint8)
    for nd in tree.leaf_node_iter():
        chars[nd.index - 1] = lut[states[nd]]
    gaps = rng.random((S, n_sites)) < gap_frac
    chars[gaps] = ord("-")
    tipcodes, weights, _ = data.compress_patterns(chars)
    pd = data.PhyloData(tree, tipcodes, weights, rooted=True)
    return pd, dict(blens=blens, freqs=FREQS.copy(), rates=rates, rs=rs, ps=ps)
