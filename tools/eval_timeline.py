"""Per-evaluation launch timeline of a class- or pattern-sweep run from a
rocprofv3 SQLite output (`rocprofv3 --kernel-trace -- python bench.py ...`).

An evaluation starts at its pmat_kernel.  For every launch position of the
evaluation (kernel order is the same in every evaluation) prints the median
duration and the median idle gap before it on the device clock, then the
median evaluation span and the share of it the GPU sat between launches.

usage: python tools/eval_timeline.py run_results.db [--skip N] [--json]
"""
import argparse
import json
import sqlite3

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--skip", type=int, default=10, help="warm-up evaluations to drop")
    ap.add_argument("--json", action="store_true")
    args = ap.parse_args()
    con = sqlite3.connect(args.db)
    ev = sorted(((n.replace("(anonymous namespace)::", "").split("(")[0], s, e)
                 for n, s, e in con.execute("select name, start, end from kernels")), key=lambda t: t[1])
    evals, cur = [], []
    for t in ev:
        if t[0].startswith("void pmat_kernel") or t[0].startswith("pmat_kernel"):
            if cur:
                evals.append(cur)
            cur = []
        if "rocclr" in t[0] or "at::native" in t[0]:
            continue
        cur.append(t)
    if cur:
        evals.append(cur)
    evals = evals[args.skip:]
    n = max(set(len(e) for e in evals), key=[len(e) for e in evals].count)
    evals = [e for e in evals if len(e) == n]
    rows = []
    for i in range(n):
        dur = np.median([(e[i][2] - e[i][1]) * 1e-3 for e in evals])
        gap = np.median([(e[i][1] - e[i - 1][2]) * 1e-3 for e in evals]) if i else 0.0
        rows.append({"pos": i, "kernel": evals[0][i][0], "us": round(float(dur), 2), "gap_before_us": round(float(gap), 2)})
    span = float(np.median([(e[-1][2] - e[0][1]) * 1e-3 for e in evals]))
    busy = sum(r["us"] for r in rows)
    gaps = sum(r["gap_before_us"] for r in rows)
    summary = {"evaluations": len(evals), "launches": n, "span_us": round(span, 1), "kernel_us": round(busy, 1),
               "gap_us": round(gaps, 1)}
    by = {}
    for r in rows:
        k = r["kernel"]
        b = by.setdefault(k, [0, 0.0, 0.0])
        b[0] += 1
        b[1] += r["us"]
        b[2] += r["gap_before_us"]
    if args.json:
        print(json.dumps({"summary": summary, "rows": rows}))
        return
    for r in rows:
        print("%3d %-40s %8.2f us  (gap %6.2f)" % (r["pos"], r["kernel"][:40], r["us"], r["gap_before_us"]))
    print()
    for k, (c, u, g) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print("%-40s x%-3d %8.1f us  gaps %6.1f us" % (k[:40], c, u, g))
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
