"""GPU: one C-ABI context over several pattern shards (phy_create_multi).

On the one-GPU box every shard sits on device 0, so the reduction is the
device-side shard sum (the RCCL all-reduce path needs distinct devices).
Everything goes through the C-ABI alone -- no torch.distributed: the rows of
the sharded context equal the single context's to rounding, per-site log
likelihoods are gathered in pattern order, and the oracle agrees.
"""
import numpy as np
import pytest

from tests import cases
from tests.test_gpu_parity import RTOL_G, RTOL_LL, _close, check_case

pytestmark = pytest.mark.gpu


def _pair(case, shards, max_draws=1):
    from phylostan_amd.engine import TreeLikelihood
    one = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C,
                         max_draws=max_draws)
    multi = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C,
                           max_draws=max_draws, devices=[0] * shards)
    return one, multi


def _rows_close(a, b):
    assert a.shape == b.shape
    for k in range(a.shape[0]):
        assert abs(a[k, 0] - b[k, 0]) <= RTOL_LL * abs(b[k, 0])
        _close(a[k, 1:], b[k, 1:], RTOL_G, "row %d" % k)


@pytest.mark.parametrize("make,shards", [(cases.fluA_case, 2), (cases.hcv_case, 2), (cases.ds1_case, 4),
                                         (lambda: cases.random_case(71, S=30, P=1000, C=3, model="GTR"), 3),
                                         (lambda: cases.random_case(72, S=25, P=777, C=2, model="HKY",
                                                                    rooted=False), 5)],
                         ids=["fluA_2", "HCV_2", "DS1_4", "rand1000_3", "unrooted777_5"])
def test_sharded_context_equals_whole(make, shards):
    case = make()
    one, multi = _pair(case, shards, max_draws=4)
    rng = np.random.default_rng(3)
    bl = case.blens[None, :] * rng.uniform(0.7, 1.3, (4, 1))
    mv = np.repeat(case.model_vec()[None], 4, axis=0)
    _rows_close(multi.evaluate_rows(bl, mv), one.evaluate_rows(bl, mv))
    # per-site log-likelihoods gathered in pattern order, and the oracle
    res = multi.evaluate(case.blens, case.model_vec(), site_ll=True)
    check_case(case, multi, res)
    # compact rows and the asynchronous pair
    one.set_output(compact=True)
    multi.set_output(compact=True)
    ref = one.evaluate_rows(bl, mv)
    multi.submit_rows(bl, mv)
    _rows_close(multi.wait_rows(), ref)


def test_sharded_context_device_buffers():
    """phy_eval_device on the sharded context: inputs and rows on device 0."""
    import torch
    case = cases.random_case(73, S=20, P=900, C=4, model="GTR")
    one, multi = _pair(case, 3, max_draws=8)
    rng = np.random.default_rng(4)
    bl = case.blens[None, :] * rng.uniform(0.7, 1.3, (8, 1))
    mv = np.repeat(case.model_vec()[None], 8, axis=0)
    d_bl = torch.tensor(bl, device="cuda:0")
    d_mv = torch.tensor(mv, device="cuda:0")
    d_out = torch.zeros((8, multi.outlen), dtype=torch.float64, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(3):  # repeated calls reuse the shards' buffers
        multi.evaluate_device(d_bl.data_ptr(), d_mv.data_ptr(), d_out.data_ptr(), 0, n_draws=8, stream=stream)
    torch.cuda.synchronize()
    _rows_close(d_out.cpu().numpy(), one.evaluate_rows(bl, mv))


def test_sharded_class_sweep_synthetic():
    """The synthetic workload (100k sites) in 4 shards, each on the class
    sweep, against the single context."""
    from phylostan_amd import synthetic
    pd, prm = synthetic.simulate(n_sites=100_000)
    case = cases.Case("syn100k", pd.tipcodes, pd.weights, pd.peel0, True, "GTR", 4, prm["blens"], prm["freqs"],
                      prm["rates"], prm["rs"], prm["ps"])
    one, multi = _pair(case, 4)
    one.set_engine("class")
    multi.set_engine("class")
    assert multi.engine() == "class"
    a = multi.evaluate(case.blens, case.model_vec(), site_ll=True)
    b = one.evaluate(case.blens, case.model_vec(), site_ll=True)
    np.testing.assert_allclose(a.site_ll, b.site_ll, rtol=RTOL_LL, atol=1e-12)
    assert abs(a.loglik - b.loglik) <= RTOL_LL * abs(b.loglik)
    _close(a.dLdP, b.dLdP, RTOL_G, "dLdP")
    _close(a.grad_blens, b.grad_blens, RTOL_G, "grad_blens")


def test_sharded_context_refusals():
    from phylostan_amd._lib import PhyloHipError
    from phylostan_amd.engine import TreeLikelihood
    case = cases.random_case(74, S=10, P=300, C=2)
    with pytest.raises(PhyloHipError):  # 3 blocks of 128 patterns, 4 shards
        TreeLikelihood(case.tipcodes, case.weights, case.peel0, True, case.model, case.C, devices=[0] * 4)
    with pytest.raises(PhyloHipError):  # devices neither all distinct nor all the same
        TreeLikelihood(case.tipcodes, case.weights, case.peel0, True, case.model, case.C, devices=[0, 0, 1])


def test_distinct_devices_rccl_branch():
    """The RCCL branch of phy_create_multi (ncclCommInitAll, one group
    ncclAllReduce of the rows, peer copies of device inputs): runs wherever
    the box has two or more GPUs -- the one-GPU box skips it, so on that box
    this branch is unverified."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two devices (the one-GPU box has one)")
    from phylostan_amd.engine import TreeLikelihood
    case = cases.hcv_case()
    one = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, max_draws=4)
    multi = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, max_draws=4,
                           devices=[0, 1])
    rng = np.random.default_rng(5)
    bl = case.blens[None, :] * rng.uniform(0.7, 1.3, (4, 1))
    mv = np.repeat(case.model_vec()[None], 4, axis=0)
    _rows_close(multi.evaluate_rows(bl, mv), one.evaluate_rows(bl, mv))
    d_bl = torch.tensor(bl, device="cuda:0")
    d_mv = torch.tensor(mv, device="cuda:0")
    d_out = torch.zeros((4, multi.outlen), device="cuda:0", dtype=torch.float64)
    multi.evaluate_device(d_bl.data_ptr(), d_mv.data_ptr(), d_out.data_ptr(), 0, n_draws=4,
                          stream=torch.cuda.current_stream(0).cuda_stream)
    torch.cuda.synchronize()
    _rows_close(d_out.cpu().numpy(), one.evaluate_rows(bl, mv))
