"""CPU: config 1 over all 42 DS1 topologies, as the reference's pipeline runs
it (examples/SConstruct:159-188 splits DS1.trees into tree{0..41}.tree and
runs `phylostan run -m JC69 --eta 0.1` on each).

tests/golden/DS1_topologies.npz (tests/golden/make_golden.py
ds1_topologies) holds, per topology, the Stan data layout from the
reference's own phylostan/utils.py and per-pattern log-likelihoods from its
scripts/phylo.py pruner.  Here: phylostan_amd.data rebuilds every layout
bit-exactly (build container only: the raw trees exist there), and the C
oracle matches every reference log-likelihood.  Polytomy resolution order is
parity-unpinned (dendropy is absent); the DS1 trees have none beyond the
trifurcating root, which the unrooted convention handles.
"""
import os

import numpy as np
import pytest

from phylostan_amd import data
from tests import cases

D = np.load(os.path.join(cases.GOLDEN, "DS1_topologies.npz"), allow_pickle=False)
NT = D["peel"].shape[0]


def test_fixture_has_every_topology_and_topology0_is_the_config1_layout():
    assert NT == 42 and sorted(D["ll_topologies"].tolist()) == list(range(42))
    g = cases.load_layout("DS1")
    assert np.array_equal(D["peel"][0], g["peel"]) and np.array_equal(D["map"][0], g["map"])
    assert np.array_equal(D["tipbits0"], g["tipbits"]) and np.array_equal(D["weights"], g["weights"])
    assert len({D["peel"][k].tobytes() + D["perm"][k].tobytes() for k in range(NT)}) > 1


def test_every_layout_matches_reference_utils(ref_examples, tmp_path):
    lines = [ln.strip() for ln in open(os.path.join(ref_examples, "DS1", "DS1.trees")) if ln.strip()]
    assert len(lines) == NT
    taxa0 = [str(t) for t in D["taxa0"]]
    for k, line in enumerate(lines):
        tf = tmp_path / ("tree%d.tree" % k)
        tf.write_text(line)
        pd = data.load(str(tf), os.path.join(ref_examples, "DS1", "DS1.nex"), rooted=False, heterochronous=False)
        perm = D["perm"][k]
        assert pd.taxa == [taxa0[i] for i in perm], k
        np.testing.assert_array_equal(pd.tipcodes, D["tipbits0"][perm], err_msg="topology %d" % k)
        np.testing.assert_array_equal(pd.weights, D["weights"])
        np.testing.assert_array_equal(np.asarray(pd.peel), D["peel"][k], err_msg="topology %d" % k)
        np.testing.assert_array_equal(np.asarray(pd.map), D["map"][k], err_msg="topology %d" % k)


@pytest.mark.parametrize("k", range(42))
def test_oracle_matches_reference_pruner(k):
    from oracle import cpu
    case = cases.ds1_topology_case(k)
    site_ref, ll_ref = cases.ds1_topology_reference(k)
    out, sl = cpu.evaluate(case.tipcodes, case.weights, case.peel0, False, 0, case.model_vec(), case.blens, 1,
                           site_ll=True)
    np.testing.assert_allclose(sl, site_ref, rtol=1e-10, atol=1e-12)
    assert abs(out[0] - ll_ref) <= 1e-10 * abs(ll_ref)
