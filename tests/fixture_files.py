"""Write a dataset's tree + alignment files from its committed layout
fixture (tests/golden/<name>_layout.npz), so the CLI can be driven end to end
where /root/reference is absent (the GPU box).

The Newick is emitted in the fixture's own child order (peel rows), so
reading it back reproduces the taxon namespace order, node numbering, peel,
map and lowers of the fixture; the FASTA repeats every pattern ``weight``
times in pattern order, so compression gives back the same patterns and
weights (distinct symbols keep ambiguous patterns distinct).
"""
import os

import numpy as np

from tests import cases

_SYM = {1: "A", 2: "C", 4: "G", 8: "T"}
_AMBIG = {3: "M", 5: "R", 9: "W", 6: "S", 10: "Y", 12: "K", 7: "V", 11: "H", 13: "D", 14: "B", 15: "-"}


def _newick(peel1, taxa, height, S):
    kids = {int(v): (int(a), int(b)) for a, b, v in peel1}
    root = int(peel1[-1][2])

    def rec(v, parent_h):
        bl = parent_h - height[v]
        if v <= S:
            s = taxa[v - 1]
        else:
            a, b = kids[v]
            s = "(%s,%s)" % (rec(a, height[v]), rec(b, height[v]))
        return s if parent_h is None else "%s:%.17g" % (s, bl)

    a, b = kids[root]
    return "(%s,%s);" % (rec(a, height[root]), rec(b, height[root]))


def _newick_trifurcating(peel1, taxa, S):
    """An unrooted fixture's tree as the reference ships it (examples/DS1/
    DS1.trees): no branch lengths, a trifurcating root (c1, x, y) where the
    resolved root row is (c1, 2S-2, root) and node 2S-2 (1-based) = (x, y) --
    reading it back and resolving the polytomy (phylostan.py:175) gives the
    fixture's node numbering again."""
    kids = {int(v): (int(a), int(b)) for a, b, v in peel1}
    root = int(peel1[-1][2])

    def rec(v):
        if v <= S:
            return taxa[v - 1]
        a, b = kids[v]
        return "(%s,%s)" % (rec(a), rec(b))

    c1, n = kids[root]
    assert n == 2 * S - 2, "the resolved root's second child must be node 2S-2 (1-based)"
    x, y = kids[n]
    return "(%s,%s,%s);" % (rec(c1), rec(x), rec(y))


def write_dataset(name, outdir, reference_form=False):
    """reference_form (unrooted datasets): the tree file in the reference's
    own form -- trifurcating root, no branch lengths (DS1.trees)."""
    d = cases.load_layout(name)
    S = d["tipbits"].shape[0]
    taxa = [str(t) for t in d["taxa"]]
    height = np.zeros(2 * S)  # 1-based node ids
    if "heights" in d:
        height[1:S + 1] = d["tip_dates"]
        height[S + 1:] = d["heights"]
    else:  # unrooted dataset: unit-ish branch lengths
        for a, b, v in d["peel"]:
            height[v] = max(height[a], height[b]) + 0.05
    tree_path = os.path.join(outdir, name + ".tree")
    with open(tree_path, "w") as fp:
        if reference_form and "heights" not in d:
            fp.write(_newick_trifurcating(d["peel"], taxa, S) + "\n")
        else:
            fp.write(_newick(d["peel"], taxa, height, S) + "\n")
    codes = d["tipbits"]
    w = d["weights"].astype(int)
    cols = np.repeat(np.arange(codes.shape[1]), w)
    aln_path = os.path.join(outdir, name + ".fa")
    with open(aln_path, "w") as fp:
        for s in range(S):
            row = "".join(_SYM.get(int(c), _AMBIG.get(int(c), "-")) for c in codes[s, cols])
            fp.write(">%s\n%s\n" % (taxa[s], row))
    return tree_path, aln_path


def write_random_dataset(outdir, seed=0, S=8, sites=60, hetero=True):
    rng = np.random.default_rng(seed)
    peel0 = cases.random_peel(S, rng)
    taxa = ["t%d_%d" % (k, k) for k in range(S)]
    height = np.zeros(2 * S)
    height[1:S + 1] = rng.uniform(0, 0.2, S) if hetero else 0.0
    for a, b, v in peel0:
        height[v + 1] = max(height[a + 1], height[b + 1]) + rng.exponential(0.1)
    tree_path = os.path.join(outdir, "rand.tree")
    with open(tree_path, "w") as fp:
        fp.write(_newick(peel0 + 1, taxa, height, S) + "\n")
    aln_path = os.path.join(outdir, "rand.fa")
    with open(aln_path, "w") as fp:
        for s in range(S):
            fp.write(">%s\n%s\n" % (taxa[s], "".join(rng.choice(list("ACGT"), sites))))
    return tree_path, aln_path
