#!/usr/bin/env python
"""Where one sweep_kernel launch spends its cycles, step by step.

Runs the fluA batched launch (8192 draws) through a PHY_STEPTIME build of
the engine (hipcc ... -DPHY_STEPTIME -o variants/steptime.so), which records
the shader clock (s_memtime) of lane 0 of every category wave of the first 64
draws at each program step, and prints, per pass, the cycles per step
averaged over those waves, grouped by step kind, plus the phase totals.
Diagnostic only: the marks themselves add a scalar load and a wait per step.

    PHYLO_HIP_AB=1 PHYLO_HIP_LIB=$PWD/variants/steptime.so python tools/steptime.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from phylostan_amd import models
    from phylostan_amd.engine import TreeLikelihood
    from tests import cases
    case = cases.fluA_case()
    n = 8192
    eng = TreeLikelihood(case.tipcodes, case.weights, case.peel0, True, "HKY", 4, max_draws=n)
    rng = np.random.default_rng(5)
    bl = case.blens[None, :] * rng.uniform(0.8, 1.25, (n, 1))
    mv = np.stack([models.model_vector(case.freqs, models.hky_exchangeabilities(5.58), case.rs, case.ps)] * n)
    for _ in range(3):
        eng.evaluate_rows(bl, mv)
    tt = np.zeros((64 * 16, 1024), dtype=np.uint64)
    rc = eng.lib.phy_debug_steptime(tt.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    info = eng.program_info()
    S = info["nsteps"]
    tt = tt.reshape(64, 16, 1024)[:, :4].astype(np.float64)  # draws x category waves
    per = []
    for trip in range(2):
        b = trip * 320
        t0, t1 = tt[..., b + 0], tt[..., b + 1]
        fw = tt[..., b + 2:b + 2 + S]
        r0, r1 = tt[..., b + 152], tt[..., b + 153]
        rv = tt[..., b + 154:b + 154 + S]
        r_end = tt[..., b + 310]
        fsteps = np.diff(np.concatenate([fw, r0[..., None]], axis=-1), axis=-1)  # forward step s duration
        rsteps = np.diff(np.concatenate([rv, r_end[..., None]], axis=-1), axis=-1)  # reverse step (nsteps-1-k)
        per.append(dict(stage_tips=(t1 - t0).mean(), fwd=(r0 - fw[..., 0]).mean(), root=(r1 - r0).mean(),
                        rev_start=(rv[..., 0] - r1).mean(), rev=(r_end - rv[..., 0]).mean(),
                        fsteps=fsteps.mean(axis=(0, 1)), rsteps=rsteps.mean(axis=(0, 1))[::-1]))
        print("block %d: stage tips %.0f, forward %.0f, root %.0f, reverse %.0f cycles" %
              (trip, per[-1]["stage_tips"], per[-1]["fwd"], per[-1]["root"], per[-1]["rev"]))
    end = tt[..., 1000]
    print("whole draw: %.0f cycles; epilogue after the last reverse %.0f" %
          ((end - tt[..., 0]).mean(), (end - tt[..., 320 + 310]).mean()))
    e0, e1, e2 = tt[..., 990], tt[..., 991], tt[..., 992]
    print("epilogue: drain %.0f, slot rows + inner products %.0f, finalize %.0f, chain rule %.0f" %
          ((e0 - tt[..., 320 + 310]).mean(), (e1 - e0).mean(), (e2 - e1).mean(), (end - e2).mean()))
    prog = eng.debug_program() if hasattr(eng, "debug_program") else None
    for trip in range(2):
        print("block %d forward cycles per step:" % trip, " ".join("%d" % v for v in per[trip]["fsteps"]))
        print("block %d reverse cycles per step (program order):" % trip,
              " ".join("%d" % v for v in per[trip]["rsteps"]))
    np.save(os.path.join(ROOT, "gpurun_out", "steptime.npy"), tt)
    _ = prog


if __name__ == "__main__":
    main()
