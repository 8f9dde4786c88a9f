"""GPU: the sharded multi-rank path on device memory.

Ranks share cuda:0 here (the box has one GPU, and RCCL wants one device
per rank), so gloo carries the all-reduce of the CUDA output tensor; each
rank evaluates its pattern shard with the HIP engine through
``ShardedLikelihood.evaluate`` on torch's current stream -- the default the
RCCL path relies on.  The reduced output must equal the single-context
evaluation of the whole alignment.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests import cases

pytestmark = pytest.mark.gpu


def _case(name):
    if name == "HCV":
        return cases.hcv_case()
    if name == "syn200k":  # the class sweep: long enough that a reduction racing the kernels would show
        from phylostan_amd import synthetic
        pd, prm = synthetic.simulate(n_sites=200_000)
        return cases.Case("syn200k", pd.tipcodes, pd.weights, pd.peel0, True, "GTR", 4, prm["blens"], prm["freqs"],
                          prm["rates"], prm["rs"], prm["ps"])
    return cases.random_case(11, S=40, P=700, C=3, model="GTR", rooted=True)


def _worker(rank, world, port, name, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from phylostan_amd.distributed import ShardedLikelihood
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case = _case(name)
        sl = ShardedLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, rank, world,
                               device=0, max_draws=2)
        dev = torch.device("cuda:0")
        blens = torch.tensor(np.stack([case.blens, case.blens * 1.2]), device=dev)
        model = torch.tensor(np.stack([case.model_vec(), case.model_vec()]), device=dev)
        out = torch.full((2, sl.outlen), float("nan"), dtype=torch.float64, device=dev)
        for _ in range(3):  # back-to-back steps on torch's default (null) stream, as a training loop issues them
            out.fill_(float("nan"))
            sl.evaluate(blens, model, out)
        res = out.cpu().numpy()
        if rank == 0:
            q.put((sl.p0, sl.p1, res))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("name,world", [("HCV", 2), ("random", 3), ("syn200k", 2)])
def test_sharded_device_allreduce_equals_whole(name, world):
    from phylostan_amd.engine import TreeLikelihood
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    p0, p1, got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert p0 == 0 and 0 < p1 < _case(name).P
    case = _case(name)
    lik = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, max_draws=2)
    for k, scale in enumerate((1.0, 1.2)):
        want = lik.evaluate_batch((case.blens * scale)[None, :], case.model_vec()[None, :])[0]
        np.testing.assert_allclose(got[k, 0], want.loglik, rtol=1e-12)
        np.testing.assert_allclose(got[k, 1:1 + len(case.blens)], want.grad_blens, rtol=1e-10,
                                   atol=1e-11 * np.abs(want.grad_blens).max())
        np.testing.assert_allclose(got[k, -16 * case.C * len(case.blens):].reshape(want.dLdP.shape), want.dLdP,
                                   rtol=1e-10, atol=1e-11 * np.abs(want.dLdP).max())
