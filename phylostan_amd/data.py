"""Data preparation for the pruning kernels (host side, no dendropy).

Restates the input-layout half of the hot path:
node numbering, peeling order, pre-order map and pattern compression, with
the reference's names and conventions so the engine can be fed exactly the
arrays phylostan's ``run()`` hands to Stan (``phylostan/phylostan.py:164-
286``).  The kernel-facing encoding differs in one way only: tips are 4-bit
state masks (A=1, C=2, G=4, T=8, anything else 15) in a ``uint8 [S, P]``
array instead of the ``int [S, L, 4]`` one-hot ``tipdata`` -- the same
information in 1/32 of the bytes.
"""
import csv

import numpy as np

from .treeio import read_alignment, read_tree

# --------------------------------------------------------------------------
# Tree indexing  (phylostan/utils.py:5-104)
# --------------------------------------------------------------------------


def get_dates(tree):
    """Root-to-tip distances (utils.py:5-16)."""
    d_internal = {}
    d_leaf = {}
    for node in tree.preorder_node_iter():
        if node.parent_node is None:
            d_internal[node] = 0
        else:
            if node.is_leaf():
                d_leaf[str(node.taxon).strip("'")] = d_internal[node.parent_node] + node.edge_length
            else:
                d_internal[node] = d_internal[node.parent_node] + node.edge_length
    return d_leaf


def setup_dates(tree, dates=None, heterochronous=False):
    """Tip dates / ages (utils.py:18-56).  Returns the oldest sample age."""
    if dates:
        heterochronous = True
    if heterochronous:
        d = {}
        if dates:
            if dates == "fasta":
                for node in tree.leaf_node_iter():
                    d[str(node.taxon).strip("'")] = float(str(node.taxon).split("_")[-1][:-1].strip("'"))
            else:
                path = getattr(dates, "name", dates)
                with open(path) as csvfile:
                    for row in csv.DictReader(csvfile):
                        d[row["name"]] = float(row["date"].strip())
        else:
            d = get_dates(tree)
        max_date = max(d.values())
        min_date = min(d.values())
        if min_date == 0:
            for node in tree.leaf_node_iter():
                node.date = d[str(node.taxon).strip("'")]
            oldest = max_date
        else:
            for node in tree.leaf_node_iter():
                node.date = max_date - d[str(node.taxon).strip("'")]
            oldest = max_date - min_date
    else:
        for node in tree.postorder_node_iter():
            node.date = 0.0
        oldest = None
    return oldest


def setup_indexes(tree):
    """Tips 1..S in taxon-namespace order, internal nodes S+1..2S-1 in
    post-order (utils.py:59-72)."""
    s = len(tree.taxon_namespace) + 1
    taxa = {t.label: i for i, t in enumerate(tree.taxon_namespace)}
    for node in tree.postorder_node_iter():
        if not node.is_leaf():
            node.index = s
            s += 1
        else:
            node.index = taxa[node.taxon.label] + 1


def get_peeling_order(tree):
    """``peel[S-1][3]`` = [child1, child2, parent], 1-based (utils.py:75-81)."""
    return [[c.index for c in node.child_node_iter()] + [node.index]
            for node in tree.postorder_node_iter() if not node.is_leaf()]


def get_preorder(tree):
    """``map[2S-1][2]`` = [node, parent] in pre-order, root row [root, 0]
    (utils.py:84-90)."""
    rows = [[tree.seed_node.index, 0]]
    for node in tree.preorder_node_iter():
        if node.parent_node is not None:
            rows.append([node.index, node.parent_node.index])
    return rows


def get_lowers(tree):
    """Lower bound of every node's height (utils.py:93-104)."""
    lowers = [0 for _ in tree.postorder_node_iter()]
    ll = {}
    for node in tree.postorder_node_iter():
        if node.is_leaf():
            ll[node] = node.date
        else:
            ll[node] = max(ll[x] for x in node.child_node_iter())
    for node in tree.preorder_node_iter():
        lowers[node.index - 1] = ll[node]
    return lowers


def unrooted_peel(peel):
    """The unrooted (no clock) convention of ``phylostan.py:264-267``: the
    last peel row lists the larger child index second, so child 2 is node
    2S-2 (1-based) whose branch is merged into child 1's."""
    peel = [list(r) for r in peel]
    last = peel[-1]
    if last[0] > last[1]:
        peel[-1] = [last[1], last[0], last[2]]
    return peel


def heights_from_tree(tree):
    """Internal node heights ``heights[S-1]`` (index node.index - S - 1) from
    the tree's branch lengths and the tip dates set by ``setup_dates``."""
    S = len(tree.taxon_namespace)
    height = {}
    for node in tree.postorder_node_iter():
        if node.is_leaf():
            height[node] = node.date
        else:
            height[node] = max(height[c] + c.edge_length for c in node.child_node_iter())
    out = np.zeros(S - 1)
    for node in tree.postorder_node_iter():
        if not node.is_leaf():
            out[node.index - S - 1] = height[node]
    return out


# --------------------------------------------------------------------------
# Pattern compression  (phylostan/utils.py:156-190)
# --------------------------------------------------------------------------
_DNA_CODE = np.full(256, 15, dtype=np.uint8)
for _ch, _code in (("A", 1), ("C", 2), ("G", 4), ("T", 8)):
    _DNA_CODE[ord(_ch)] = _code
    _DNA_CODE[ord(_ch.lower())] = _code


def alignment_matrix(alignment, taxon_namespace):
    """Rows of the alignment in taxon-namespace order (DendroPy iterates a
    CharacterMatrix in namespace order) as a ``uint8 [S, sites]`` char array."""
    rows = []
    for taxon in taxon_namespace:
        label = taxon.label if hasattr(taxon, "label") else taxon
        rows.append(np.frombuffer(alignment[label].upper().encode("ascii"), dtype=np.uint8))
    n = {len(r) for r in rows}
    if len(n) != 1:
        raise ValueError("alignment rows have different lengths: %s" % sorted(n))
    return np.stack(rows)


def compress_patterns(chars):
    """Site-pattern compression of ``get_dna_leaves_partials_compressed``
    (utils.py:156-190), vectorised.

    ``chars``: ``uint8 [S, sites]`` (upper-case symbols).  Columns are
    deduplicated on their raw symbols, kept in order of first occurrence, and
    weighted by multiplicity.  Returns ``(tipcodes uint8 [S, P], weights
    float64 [P], first_site int64 [P])``.
    """
    chars = np.ascontiguousarray(chars, dtype=np.uint8)
    S, n_sites = chars.shape
    cols = np.ascontiguousarray(chars.T)
    view = cols.view(np.dtype((np.void, S)))[:, 0]
    _, first, inverse, counts = np.unique(view, return_index=True, return_inverse=True,
                                          return_counts=True)
    order = np.argsort(first, kind="stable")
    first_sorted = first[order]
    weights = counts[order].astype(np.float64)
    tipcodes = _DNA_CODE[chars[:, first_sorted]]
    return tipcodes, weights, first_sorted


def codes_to_tipdata(tipcodes):
    """``uint8 [S, P]`` masks -> the reference's ``tipdata[S][P][4]`` 0/1."""
    return ((tipcodes[..., None] >> np.arange(4)) & 1).astype(np.int64)


# --------------------------------------------------------------------------
# The Stan data dict of phylostan.run()  (phylostan.py:164-286)
# --------------------------------------------------------------------------
class PhyloData:
    """Everything the likelihood needs, in the reference's conventions.

    Attributes (1-based, as in the Stan data dict): ``peel``, ``map``,
    ``lowers``; kernel-facing: ``tipcodes [S, P]``, ``weights [P]``,
    ``peel0`` (0-based), ``rooted``.
    """

    def __init__(self, tree, tipcodes, weights, rooted, heterochronous=False, oldest=None):
        self.tree = tree
        self.S = len(tree.taxon_namespace)
        self.tipcodes = tipcodes
        self.weights = weights
        self.P = tipcodes.shape[1]
        self.rooted = rooted
        peel = get_peeling_order(tree)
        self.peel = peel if rooted else unrooted_peel(peel)
        self.peel0 = np.asarray(self.peel, dtype=np.int32) - 1
        self.map = get_preorder(tree)
        self.lowers = get_lowers(tree) if heterochronous else None
        self.oldest = oldest
        self.B = 2 * self.S - 2 if rooted else 2 * self.S - 3

    @property
    def taxa(self):
        return [t.label for t in self.tree.taxon_namespace]


def load(tree_path, alignment_path, rooted=True, heterochronous=False, dates=None):
    """Read + index + compress exactly as ``phylostan.run`` does
    (phylostan.py:172-204, :255-267)."""
    tree = read_tree(tree_path)
    tree.resolve_polytomies(update_bipartitions=True)
    setup_indexes(tree)
    oldest = setup_dates(tree, dates, heterochronous)
    aln = read_alignment(alignment_path)
    missing = [t.label for t in tree.taxon_namespace if t.label not in aln]
    if missing or len(aln) != len(tree.taxon_namespace):
        raise ValueError("taxon names in trees and alignment are different: %s" % missing[:5])
    chars = alignment_matrix(aln, tree.taxon_namespace)
    tipcodes, weights, _ = compress_patterns(chars)
    return PhyloData(tree, tipcodes, weights, rooted, heterochronous, oldest)
