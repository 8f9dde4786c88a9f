"""GPU: phy_eval_device with stream = NULL is ordered with the caller's legacy
null stream.

torch's default stream is HIP's null stream (handle 0).  A producer on it
(the inputs' copies), phy_eval_device(..., NULL), then a consumer on it (a
clone of the rows) -- with no synchronisation of the caller's own -- must
see exactly the rows a synchronous phy_eval returns.  Before the fence the
engine ran on its own non-blocking stream and a consumer could read rows not
yet written (the N = 2 rehearsal's nominal check, r05).  The reference's
boundary is one synchronous call (eigen/prune_stan.hpp:9-17).
"""
import numpy as np
import pytest

from tests import cases

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shards", [0, 2], ids=["single_context", "two_shard_context"])
def test_eval_device_on_the_null_stream_is_ordered_with_it(shards):
    import torch
    from phylostan_amd import models
    from phylostan_amd.engine import TreeLikelihood
    case = cases.fluA_case()
    n = 256  # above the pinned small-call path: phy_eval runs the same launches as phy_eval_device
    eng = TreeLikelihood(case.tipcodes, case.weights, case.peel0, True, "HKY", 4, max_draws=n,
                         devices=[0] * shards if shards else None)
    dev = torch.device("cuda:0")
    assert torch.cuda.current_stream(dev).cuda_stream == 0  # the test runs on the null stream
    rng = np.random.default_rng(17)
    d_bl = torch.empty((n, eng.B), dtype=torch.float64, device=dev)
    d_mv = torch.empty((n, eng.model_len), dtype=torch.float64, device=dev)
    d_out = torch.empty((n, eng.outlen), dtype=torch.float64, device=dev)
    for it in range(6):
        blens = case.blens[None, :] * rng.uniform(0.6, 1.4, (n, eng.B))
        mvs = np.stack([models.model_vector(case.freqs, models.hky_exchangeabilities(rng.uniform(3.0, 8.0)),
                                            case.rs, case.ps) for _ in range(n)])
        ref = eng.evaluate_rows(blens, mvs)  # phy_eval: synchronous, host buffers
        h_bl = torch.from_numpy(blens).pin_memory()
        h_mv = torch.from_numpy(mvs).pin_memory()
        # producer on the null stream: asynchronous uploads, then a poisoned output
        d_bl.copy_(h_bl, non_blocking=True)
        d_mv.copy_(h_mv, non_blocking=True)
        d_out.fill_(float("nan"))
        eng.evaluate_device(d_bl.data_ptr(), d_mv.data_ptr(), d_out.data_ptr(), n_draws=n, stream=0)
        # consumer on the null stream, no synchronisation in between
        got = d_out.clone()
        d_out.fill_(float("nan"))  # a later writer on the null stream must not race the engine either
        rows = got.cpu().numpy()
        assert np.array_equal(rows, ref), "iteration %d: rows differ from the synchronous phy_eval" % it
