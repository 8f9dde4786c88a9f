#!/usr/bin/env python
"""Two contexts, phy_eval_submit / phy_eval_wait: does one context's
evaluation overlap the other's?  Prints us per evaluation for one context
(submit + wait) and for two interleaved contexts (submit A, submit B, wait A,
wait B)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from phylostan_amd.engine import TreeLikelihood
    from tests import cases
    eng = sys.argv[1] if len(sys.argv) > 1 else "pattern"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    case = cases.fluA_case()
    liks = []
    for _ in range(2):
        lk = TreeLikelihood(case.tipcodes, case.weights, case.peel0, True, case.model, case.C, max_draws=n)
        lk.set_output(compact=True)
        lk.set_engine(eng)
        liks.append(lk)
    bl = np.stack([case.blens * (1.0 + 0.01 * k) for k in range(n)])
    mv = np.stack([case.model_vec()] * n)
    calls = 300
    for lk in liks:
        for _ in range(10):
            lk.submit_rows(bl, mv)
            lk.wait_rows()
    t0 = time.perf_counter()
    for _ in range(calls):
        liks[0].submit_rows(bl, mv)
        liks[0].wait_rows()
    one = (time.perf_counter() - t0) / calls
    t0 = time.perf_counter()
    for _ in range(calls):
        liks[0].submit_rows(bl, mv)
        liks[1].submit_rows(bl, mv)
        liks[0].wait_rows()
        liks[1].wait_rows()
    two = (time.perf_counter() - t0) / (2 * calls)
    print(json.dumps({"engine": eng, "draws": n, "us_per_eval_one_ctx": one * 1e6,
                      "us_per_eval_two_ctx_interleaved": two * 1e6}))


if __name__ == "__main__":
    main()
