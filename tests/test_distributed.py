"""CPU: the N>1 path -- pattern shards + one all-reduce (gloo, world size 2).

ShardedLikelihood is the product's multi-GPU layer (one process per GPU,
RCCL on the box).  Here each rank evaluates its shard with the C oracle
(test infrastructure) behind the same device-pointer interface, and the
all-reduced output vector must equal the single-process evaluation.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from phylostan_amd.distributed import ShardedLikelihood, shard_range
from tests import cases


class OracleShardEngine:
    """Shard evaluator with the TreeLikelihood.evaluate_device contract,
    computing on the CPU with oracle/cpu_pruner.c (tests only)."""

    def __init__(self, tipcodes, weights, peel0, rooted, model, C, max_draws=1, device=0):
        from oracle import numpy_pruner as npr
        self.args = (tipcodes, weights, peel0, rooted, npr.MODEL_IDS[model], C)
        S = tipcodes.shape[0]
        self.B = 2 * S - 2 if rooted else 2 * S - 3
        self.C = C
        self.outlen = 1 + self.B + 2 * C + 4 + 10 + 16 * C * self.B

    def set_output(self, compact=False):
        """compact rows: the full row without its dL/dP block (phy_set_output)."""
        self.outlen = 1 + self.B + 2 * self.C + 4 + 10 + (0 if compact else 16 * self.C * self.B)

    def evaluate_device(self, d_blens, d_model, d_out, d_site_ll=0, n_draws=1, stream=0):
        from oracle import cpu
        tip, w, peel, rooted, kind, C = self.args
        ml = 10 + 2 * C
        for k in range(n_draws):
            bl = np.ctypeslib.as_array((ctypes.c_double * self.B).from_address(d_blens + 8 * k * self.B)).copy()
            mv = np.ctypeslib.as_array((ctypes.c_double * ml).from_address(d_model + 8 * k * ml)).copy()
            out, _ = cpu.evaluate(tip, w, peel, rooted, kind, mv, bl, C)
            ctypes.memmove(d_out + 8 * k * self.outlen, out.ctypes.data, 8 * self.outlen)


def _worker(rank, world, port, case_args, result_q, compact=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    case = cases.random_case(*case_args[0], **case_args[1])
    sl = ShardedLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C,
                           rank, world, max_draws=2, engine_factory=OracleShardEngine, compact=compact)
    blens = torch.tensor(np.stack([case.blens, case.blens * 1.3]))
    model = torch.tensor(np.stack([case.model_vec(), case.model_vec()]))
    out = torch.zeros((2, sl.outlen), dtype=torch.float64)
    sl.evaluate(blens, model, out)
    if rank == 0:
        result_q.put(out.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_sharded(world, case_args, compact):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case_args, q, compact)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world", [2])
def test_sharded_allreduce_equals_full(world):
    case_args = ((4,), dict(S=11, P=97, C=3, model="GTR", rooted=True))
    got = _run_sharded(world, case_args, compact=False)
    case = cases.random_case(*case_args[0], **case_args[1])
    eng = OracleShardEngine(case.tipcodes, case.weights, case.peel0, True, case.model, case.C)
    for k, scale in enumerate((1.0, 1.3)):
        from oracle import cpu
        full, _ = cpu.evaluate(case.tipcodes, case.weights, case.peel0, True, 2, case.model_vec(),
                               case.blens * scale, case.C)
        np.testing.assert_allclose(got[k], full, rtol=1e-11, atol=1e-11 * np.abs(full).max())
    assert eng.outlen == got.shape[1]


def test_sharded_compact_allreduce_equals_compact_rows_of_full_sum():
    """The sampler's collective (compact rows: log-lik and every parameter
    gradient, no dL/dP block -- 2.2 KB instead of 132 KB per draw at the
    synthetic config): the all-reduced compact rows of two pattern shards
    equal the compact part of the all-reduced full rows, and the whole
    alignment's rows.  The exchangeability / frequency gradients are linear
    in dL/dP and the root term, so they sum across shards like the rest."""
    case_args = ((4,), dict(S=11, P=97, C=3, model="GTR", rooted=True))
    full = _run_sharded(2, case_args, compact=False)
    comp = _run_sharded(2, case_args, compact=True)
    case = cases.random_case(*case_args[0], **case_args[1])
    B, C = 2 * case.tipcodes.shape[0] - 2, case.C
    G = 1 + B + 2 * C + 14
    assert comp.shape == (2, G) and full.shape[1] == G + 16 * C * B
    np.testing.assert_allclose(comp, full[:, :G], rtol=1e-13, atol=1e-13 * np.abs(full[:, :G]).max())
    from oracle import cpu
    for k, scale in enumerate((1.0, 1.3)):
        whole, _ = cpu.evaluate(case.tipcodes, case.weights, case.peel0, True, 2, case.model_vec(),
                                case.blens * scale, case.C)
        np.testing.assert_allclose(comp[k], whole[:G], rtol=1e-11, atol=1e-11 * np.abs(whole[:G]).max())


def test_shard_ranges_cover_and_balance():
    for P in (1, 7, 238, 528111):
        for world in (1, 2, 3, 8):
            if P < world:
                continue
            rs = [shard_range(P, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == P
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [b - a for a, b in rs]
            assert min(sizes) >= 1
            if -(-P // 128) >= world:  # whole 128-pattern sweep blocks per rank
                assert all(a % 128 == 0 for a, _ in rs)
                blocks = [-(-(b - a) // 128) for a, b in rs]
                assert max(blocks) - min(blocks) <= 1
            else:
                assert max(sizes) - min(sizes) <= 1


def test_bench_spawns_one_rank_per_gpu():
    """``python bench.py --gpus 2`` with no launcher starts two ranks through
    torch.distributed.run (the driver's N>1 command); --dry-run stops after
    the ranks joined a gloo group, before anything touches a GPU."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    rec = json.loads(line)
    assert rec == {"dry_run": True, "n_gpus": 2, "sum_of_ranks": 1}
    env["WORLD_SIZE"] = "3"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
