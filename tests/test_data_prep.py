"""CPU: the host data layer against the reference's own data layout.

The golden layouts (tests/golden/<dataset>_layout.npz) were produced by the
reference's phylostan/utils.py functions (setup_indexes, setup_dates,
get_peeling_order, get_preorder, get_lowers, get_dna_leaves_partials_
compressed) run on the example inputs -- see tests/golden/make_golden.py.
Rebuilding the layout with phylostan_amd.data must give identical arrays.
The raw inputs exist only in the build container (the GPU box has no
/root/reference): those tests skip there.
"""
import os

import numpy as np
import pytest

from phylostan_amd import data, treeio
from tests import cases

DATASETS = {
    "fluA": ("fluA/fluA.tree", "fluA/fluA.fa", True, True),
    "HCV": ("HCV/HCV.tree", "HCV/HCV.nexus", False, True),
    "DS1": ("DS1/DS1.trees", "DS1/DS1.nex", False, False),
}


@pytest.mark.parametrize("name", sorted(DATASETS))
def test_layout_matches_reference_utils(name, ref_examples):
    tpath, apath, het, rooted = DATASETS[name]
    pd = data.load(os.path.join(ref_examples, tpath), os.path.join(ref_examples, apath),
                   rooted=rooted, heterochronous=het)
    g = cases.load_layout(name)
    assert pd.taxa == list(g["taxa"])
    np.testing.assert_array_equal(pd.tipcodes, g["tipbits"])
    np.testing.assert_array_equal(pd.weights, g["weights"])
    np.testing.assert_array_equal(np.asarray(pd.peel), g["peel"])
    np.testing.assert_array_equal(np.asarray(pd.map), g["map"])
    assert pd.weights.sum() == g["sites"]
    if het:
        np.testing.assert_allclose(pd.lowers, g["lowers"], rtol=0, atol=0)


def test_golden_pattern_counts():
    """Pattern counts recorded in SURVEY.md 2 (examples row)."""
    for name, P in (("fluA", 238), ("HCV", 246), ("DS1", 934)):
        g = cases.load_layout(name)
        assert g["tipbits"].shape[1] == P


def test_compress_patterns_first_seen_order():
    chars = np.array([list(b"ACGTA-"), list(b"ACGTA-"), list(b"ACNTAC")], dtype=np.uint8)
    codes, w, first = data.compress_patterns(chars)
    # columns 0 and 4 are identical (A,A,A)
    np.testing.assert_array_equal(first, [0, 1, 2, 3, 5])
    np.testing.assert_array_equal(w, [2, 1, 1, 1, 1])
    assert codes[2, 2] == 15  # 'N' -> all ones (utils.py:187)
    assert codes[0, 4] == 15 and codes[2, 4] == 2  # '-' -> all ones, C
    td = data.codes_to_tipdata(codes)
    assert td.shape == (3, 5, 4) and td[0, 0].tolist() == [1, 0, 0, 0]


def test_compress_distinguishes_ambiguity_symbols():
    """utils.py:163-165 dedups on raw symbols: 'N' and '-' are different
    patterns even though both encode to [1,1,1,1]."""
    chars = np.array([list(b"N-"), list(b"AA")], dtype=np.uint8)
    codes, w, _ = data.compress_patterns(chars)
    assert codes.shape[1] == 2 and np.all(codes[0] == 15)


def test_compress_large_random_sums_to_sites():
    rng = np.random.default_rng(0)
    chars = rng.choice(np.frombuffer(b"ACGT-", dtype=np.uint8), size=(12, 5000), p=[.3, .2, .2, .29, .01])
    chars[:, 100:200] = chars[:, 0:1]
    codes, w, first = data.compress_patterns(chars)
    assert w.sum() == 5000
    assert np.all(np.diff(first) > 0)
    rebuilt = codes[:, np.searchsorted(first, first)]
    assert rebuilt.shape == codes.shape


def test_newick_parser_conventions():
    t = treeio.parse_newick("(('a b':1,[&x=1]B_c:2)n1:0.5,C:3,D:1e-2)root;")
    labels = [x.label for x in t.taxon_namespace]
    assert labels == ["a b", "B_c", "C", "D"]  # file order, quotes removed, underscores kept
    t.resolve_polytomies()
    assert all(len(n.child_nodes()) in (0, 2) for n in t.postorder_node_iter())
    data.setup_indexes(t)
    peel = data.get_peeling_order(t)
    assert peel[-1][2] == 2 * 4 - 1  # root is 2S-1
    assert sorted(n.index for n in t.postorder_node_iter()) == list(range(1, 8))
    m = data.get_preorder(t)
    assert m[0] == [7, 0] and len(m) == 7


def test_unrooted_peel_convention():
    peel = [[1, 2, 5], [3, 4, 6], [6, 5, 7]]
    assert data.unrooted_peel(peel)[-1] == [5, 6, 7]


def test_clock_blens_matches_reference_formula():
    """blens[node] = rate * (h[parent] - h[node]) (generate_script.py:660-679)."""
    g = cases.load_layout("fluA")
    S = g["tipbits"].shape[0]
    peel0 = g["peel"] - 1
    bl = __import__("phylostan_amd.models", fromlist=["x"]).clock_blens(g["heights"], g["tip_dates"], peel0, S, 0.5)
    h = np.concatenate([g["tip_dates"], g["heights"]])
    for node, parent in g["map"][1:]:
        assert abs(bl[node - 1] - 0.5 * (h[parent - 1] - h[node - 1])) < 1e-12
    assert np.all(bl > 0)
