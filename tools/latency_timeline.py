"""Per-call timeline of a sampler-shaped call from a rocprofv3 SQLite output
(`rocprofv3 --kernel-trace --memory-copy-trace -- python tools/latency_probe.py ...`).

A call is the H2D copy of its inputs through the D2H copy of its rows (small
copies from pinned memory run as `__amd_rocclr_copyBuffer` blit kernels: a
call starts at a blit whose next activity is `pmat_kernel`).  Prints
one JSON object: the median of each kernel's and copy's duration, the median
call span (first copy start to last copy end on the device clock), and the
span not covered by any device activity (launch and copy gaps).

usage: python tools/latency_timeline.py run_results.db [--skip N]
"""
import argparse
import json
import sqlite3
from collections import defaultdict

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--skip", type=int, default=50, help="warm-up calls to drop")
    args = ap.parse_args()
    con = sqlite3.connect(args.db)
    ev = [("K", n.replace("(anonymous namespace)::", "").split("(")[0], s, e)
          for n, s, e in con.execute("select name, start, end from kernels")]
    ev += [("C", n, s, e) for n, s, e in con.execute("select name, start, end from memory_copies")]
    ev.sort(key=lambda t: t[2])

    def is_copy(t):
        return t[0] == "C" or "copyBuffer" in t[1]

    calls, cur = [], []
    for i, t in enumerate(ev):
        starts = is_copy(t) and i + 1 < len(ev) and ev[i + 1][1].startswith("pmat_kernel")
        if starts and cur:
            calls.append(cur)
            cur = []
        cur.append(t)
    if cur:
        calls.append(cur)
    calls = [c for c in calls if is_copy(c[0]) and is_copy(c[-1])][args.skip:]
    dur = defaultdict(list)
    span, busy = [], []
    for c in calls:
        for kind, name, s, e in c:
            dur[name].append((e - s) / 1e3)
        span.append((c[-1][3] - c[0][2]) / 1e3)
        busy.append(sum(e - s for _, _, s, e in c) / 1e3)
    out = {
        "calls": len(calls),
        "median_us": {k: round(float(np.median(v)), 2) for k, v in dur.items()},
        "per_call": {k: len(v) / len(calls) for k, v in dur.items()},
        "median_span_us": round(float(np.median(span)), 2),
        "median_device_busy_us": round(float(np.median(busy)), 2),
        "median_gaps_us": round(float(np.median(np.array(span) - np.array(busy))), 2),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
