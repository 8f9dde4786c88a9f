#!/usr/bin/env python
"""Summarise a PHY_FLOW_TRACE file (the class sweep's dataflow launch,
cls_flow_kernel): per launch, the span on the device's wall clock (100 MHz),
per item kind the count, mean wait for its inputs and mean work, and a
timeline of item completions.  Diagnostics only (no GPU needed to read).

    PHY_FLOW_TRACE=/tmp/ft.bin python bench.py --workload synthetic --shard-of 8 --steps 3 --warmup 1 ...
    python tools/flow_trace.py /tmp/ft.bin
"""
import sys

import numpy as np

KINDS = ["FWD", "ROOT", "RED", "FIX", "REV"]
TICK_US = 0.01  # wall_clock64 at 100 MHz


def records(path):
    raw = open(path, "rb").read()
    off = 0
    while off < len(raw):
        nitems, n, grid, isz = np.frombuffer(raw, np.int32, 4, off)
        off += 16
        items = np.frombuffer(raw, np.int32, nitems * isz // 4, off).reshape(nitems, isz // 4)
        off += nitems * isz
        tr = np.frombuffer(raw, np.uint64, 4 * nitems * n, off).reshape(nitems * n, 4)
        off += 32 * nitems * n
        yield int(nitems), int(n), int(grid), items, tr


def main():
    recs = list(records(sys.argv[1]))
    nitems, n, grid, items, tr = recs[-1]  # the last launch (warm)
    t0 = tr[:, 0].astype(np.int64)
    t1 = tr[:, 1].astype(np.int64)
    t2 = tr[:, 2].astype(np.int64)
    base = t0.min()
    span = (t2.max() - base) * TICK_US
    kind = np.repeat(items[:, 0], n)
    print("launches %d; last: %d items x %d draws, grid %d, span %.1f us" % (len(recs), nitems, n, grid, span))
    for k, name in enumerate(KINDS):
        m = kind == k
        if not m.any():
            continue
        w = (t1[m] - t0[m]) * TICK_US
        d = (t2[m] - t1[m]) * TICK_US
        print("  %-4s %6d items  wait mean %7.2f max %7.2f us  work mean %6.2f max %6.2f us  done %7.1f..%7.1f us"
              % (name, m.sum(), w.mean(), w.max(), d.mean(), d.max(), (t2[m].min() - base) * TICK_US,
                 (t2[m].max() - base) * TICK_US))
    # per-workgroup busy time and first start
    wg = (tr[:, 3] >> np.uint64(32)).astype(np.int64)
    busy = np.bincount(wg, weights=(t2 - t1) * TICK_US)
    waits = np.bincount(wg, weights=(t1 - t0) * TICK_US)
    print("  per workgroup: work %.1f us mean (max %.1f), waiting %.1f us mean (max %.1f)"
          % (busy.mean(), busy.max(), waits.mean(), waits.max()))
    gaps = []
    for g in range(grid):
        sel = np.nonzero(wg == g)[0]
        if len(sel) > 1:
            gaps.append(((t0[sel[1:]] - t2[sel[:-1]]) * TICK_US).mean())
    if gaps:
        print("  between a workgroup's items (signal -> next wait start): %.2f us mean" % np.mean(gaps))
    edges = np.arange(0, span + 10, 10)
    print("  completions per 10 us:", " ".join("%d" % c for c in np.histogram((t2 - base) * TICK_US, edges)[0]))


if __name__ == "__main__":
    main()
