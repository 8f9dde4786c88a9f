#!/usr/bin/env python
"""Small-batch latency of one log-lik + gradient evaluation (the NUTS round
shape: n draws per call, compact rows, host buffers): wall time per call.
Run on the GPU box, optionally under rocprofv3 --kernel-trace --stats."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--draws", type=int, default=4)
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--workload", default="fluA", choices=["fluA", "HCV", "DS1"])
    ap.add_argument("--engine", default="auto", choices=["auto", "pattern", "class"])
    ap.add_argument("--cols", type=int, default=0, help="pattern columns per lane (0 = the plan's choice)")
    ap.add_argument("--lds-budget", type=int, default=0)
    a = ap.parse_args()
    from phylostan_amd.engine import TreeLikelihood
    from tests import cases
    case = {"fluA": cases.fluA_case, "HCV": cases.hcv_case, "DS1": cases.ds1_case}[a.workload]()
    lik = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C,
                         max_draws=a.draws)
    lik.set_output(compact=True)
    if a.engine != "auto":
        lik.set_engine(a.engine)
    if a.cols or a.lds_budget:
        lik.set_tuning(cols=a.cols, lds_budget=a.lds_budget)
    bl = np.stack([case.blens * (1.0 + 0.01 * k) for k in range(a.draws)])
    mv = np.stack([case.model_vec()] * a.draws)
    for _ in range(20):
        lik.evaluate_rows(bl, mv)
    t0 = time.perf_counter()
    for _ in range(a.calls):
        lik.evaluate_rows(bl, mv)
    dt = (time.perf_counter() - t0) / a.calls
    print(json.dumps({"workload": a.workload, "engine": lik.engine(), "draws": a.draws, "cols": a.cols,
                      "lds_budget": a.lds_budget, "us_per_call": dt * 1e6}))


if __name__ == "__main__":
    main()
