#!/usr/bin/env python
"""Where the class sweep's epilogue spends its time.

Runs the synthetic workload (the first of --shard-of N pattern shards, or the
whole alignment) through a PHY_EPITIME build of the engine
(hipcc ... -DPHY_EPITIME -o variants/epitime.so), which records the GPU
real-time clock (s_memrealtime, 100 MHz) of wave 0 of every epilogue
workgroup of draw 0 at its phase boundaries -- per-item launch: 0 start,
1 chunk-partial sums in LDS, 2 hand-offs stored; closing launch (last row):
0 start, 3 M summed (wave 0), 7 branch sums, 4 barrier, 5 per-category sums
done, 6 Q-parameter tail done.  Prints the phase durations (median / 90th percentile over the
workgroups), how the workgroup starts spread over the launch, and the
closing workgroup's timeline.  Diagnostic only.

    PHYLO_HIP_AB=1 PHYLO_HIP_LIB=$PWD/variants/epitime.so python tools/epitime.py --shard-of 8
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard-of", type=int, default=8)
    ap.add_argument("--sites", type=int, default=1_000_000)
    a = ap.parse_args()
    import torch
    import bench
    from phylostan_amd.distributed import ShardedLikelihood
    prob = bench.synthetic_problem(a.sites)
    sl = ShardedLikelihood(prob["tipcodes"], prob["weights"], prob["peel0"], prob["rooted"], prob["model"],
                           prob["C"], 0, max(1, a.shard_of), device=0, max_draws=1)
    eng = sl.engine
    rng = np.random.default_rng(1)
    blens, mvs = bench.parameter_sets(prob, 4, 1, eng.B, prob["C"], rng)
    dev = torch.device("cuda:0")
    d_bl = torch.tensor(blens, device=dev, dtype=torch.float64)
    d_mv = torch.tensor(mvs, device=dev, dtype=torch.float64)
    d_out = torch.zeros((1, eng.outlen), device=dev, dtype=torch.float64)
    st = torch.cuda.Stream(device=dev)
    for k in range(20):
        eng.evaluate_device(d_bl[k % 4].data_ptr(), d_mv[k % 4].data_ptr(), d_out.data_ptr(), 0, n_draws=1,
                            stream=st.cuda_stream)
    torch.cuda.synchronize(dev)
    et = np.zeros((4096, 8), dtype=np.uint64)
    assert eng.lib.phy_debug_epitime(et.ctypes.data_as(ctypes.c_void_p)) == 0
    ni = prob["C"] * eng.B
    t = et.astype(np.float64) * 10.0 / 1000.0  # 100 MHz ticks -> us
    close = t[-1]
    t = t[:ni]
    t0 = t[:, 0].min()
    t, close = t - t0, close - t0
    print("items %d" % ni)
    for name, a0, a1 in (("start -> partial sums", 0, 1), ("partial sums -> hand-offs stored", 1, 2)):
        d = t[:, a1] - t[:, a0]
        print("  %-36s median %6.2f us  p90 %6.2f  max %6.2f" % (name, np.median(d), np.percentile(d, 90), d.max()))
    s = np.sort(t[:, 0])
    print("  workgroup starts: first %.2f, 25%% %.2f, 50%% %.2f, 75%% %.2f, last %.2f us" %
          (s[0], s[len(s) // 4], s[len(s) // 2], s[3 * len(s) // 4], s[-1]))
    print("  last hand-off stored %.2f us" % t[:, 2].max())
    print("  closing workgroup: start %.2f, M summed %.2f, branch sums %.2f, barrier %.2f, per-category %.2f, "
          "tail %.2f us" % (close[0], close[3], close[7], close[4], close[5], close[6]))
    np.save(os.path.join(ROOT, "gpurun_out", "epitime.npy"), t)


if __name__ == "__main__":
    main()
