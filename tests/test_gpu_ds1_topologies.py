"""GPU: config 1 on all 42 DS1 topologies (examples/SConstruct:159-188 runs
`phylostan run -m JC69` on every line of DS1.trees) through the C-ABI, on
every engine: the quad sweep (a sampler's 4-draw call), the column sweep (a
batched 64-draw launch) and the class sweep -- every per-site
log-likelihood against the reference's scripts/phylo.py values
(tests/golden/DS1_topologies.npz) at rel 1e-10, and every output row against
the C oracle at the parity bar of tests/test_gpu_parity.py."""
import numpy as np
import pytest

from tests import cases
from tests.test_gpu_parity import RTOL_G, RTOL_LL, _close, check_case

pytestmark = pytest.mark.gpu


def _rows_vs_oracle(rows, case):
    from oracle import cpu
    ref, _ = cpu.evaluate(case.tipcodes, case.weights, case.peel0, False, 0, case.model_vec(), case.blens, 1)
    for r in rows:
        assert abs(r[0] - ref[0]) <= RTOL_LL * abs(ref[0])
        _close(r[1:len(ref)], ref[1:], RTOL_G, "row")


@pytest.mark.parametrize("k", range(42))
def test_ds1_topology_every_engine(k):
    from phylostan_amd.engine import TreeLikelihood
    case = cases.ds1_topology_case(k)
    site_ref, ll_ref = cases.ds1_topology_reference(k)
    lines = []
    for engine, n in (("pattern", 4), ("pattern", 64), ("class", 4)):
        eng = TreeLikelihood(case.tipcodes, case.weights, case.peel0, False, "JC69", 1, max_draws=n)
        eng.set_engine(engine)
        res = check_case(case, eng)  # one draw with site log-likelihoods, against the oracle
        np.testing.assert_allclose(res.site_ll, site_ref, rtol=RTOL_LL, atol=1e-12)
        assert abs(res.loglik - ll_ref) <= RTOL_LL * abs(ll_ref)
        rows = eng.evaluate_rows(np.repeat(case.blens[None], n, axis=0), np.repeat(case.model_vec()[None], n, axis=0))
        _rows_vs_oracle(rows, case)
        lines.append("%s/%d" % (engine, n))
        eng.close()
    assert len(lines) == 3
