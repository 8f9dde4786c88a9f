#!/usr/bin/env python
"""Per-kernel statistics from a rocprofv3 SQLite output (``rocprofv3
--kernel-trace --stats -d DIR -o run``): calls, total / average / min / max
duration, share -- the columns of rocprofv3's kernel_stats.csv -- plus the
average GPU-side gap between consecutive dispatches.

    python tools/prof_stats.py DIR/run_results.db [--csv OUT.csv] [--filter SUBSTR]
"""
import argparse
import csv
import sqlite3
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0] if "(" in name else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = [(n, s, e) for n, s, e in con.execute("select name, start, end from kernels order by start")]
    rows = [r for r in rows if a.filter in r[0]]
    st = defaultdict(list)
    for n, s, e in rows:
        st[n].append(e - s)
    tot = sum(sum(v) for v in st.values()) or 1
    out = []
    for n, v in sorted(st.items(), key=lambda kv: -sum(kv[1])):
        out.append([n, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)])
    gaps = [rows[i + 1][1] - rows[i][2] for i in range(len(rows) - 1) if rows[i + 1][1] > rows[i][2]]
    w = sys.stdout
    for r in out:
        w.write("%-60s %6d %12d %10.1f %6.2f%% %8d %8d\n" % (short(r[0])[:60], r[1], r[2], r[3], r[4], r[5], r[6]))
    if gaps:
        w.write("dispatches %d, mean gap between consecutive dispatches %.1f ns\n" % (len(rows), sum(gaps) / len(gaps)))
    if a.csv:
        with open(a.csv, "w", newline="") as fp:
            cw = csv.writer(fp, quoting=csv.QUOTE_NONNUMERIC)
            cw.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for r in out:
                cw.writerow(r)


if __name__ == "__main__":
    main()
