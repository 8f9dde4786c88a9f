#!/usr/bin/env python
"""Collect the sweep kernel's HBM traffic with rocprofv3 PMC counters and
record it for bench.py's roofline.traffic field.

Run ON THE GPU BOX (it launches rocprofv3 as a child process; this script
never touches the GPU itself):
    python tools/pmc_traffic.py [--workload fluA|synthetic] [--draws N]

Two separate passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass),
--kernel-trace only, as MI355X_MICROARCH.md "HBM" prescribes.  gfx950
correction: FETCH_SIZE reports half the bytes of a 16-B-per-lane coalesced
read, so traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes per dispatch
(averaged over the sweep_kernel dispatches of the run).  Results are keyed
by the kernel source hash, so a stale record is never reported.
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


# the class sweep's timed region (phy_timing_*: forward through the last reverse level)
CLASS_KERNELS = ("cls_clade_fwd_kernel", "cls_fwd_kernel", "cls_fwd2_kernel", "cls_chain_fwd_kernel", "cls_root_kernel", "cls_red_kernel",
                 "cls_red_list_kernel", "cls_fix_list_kernel", "cls_rev_kernel", "cls_rev_ls_kernel", "cls_chain_rev_kernel",
                 "cls_clade_rev_kernel")


def run_pass(counter, out_dir, bench_args, engine):
    """Average per launch of the timed region: the sweep_kernel dispatch
    (pattern sweep) or the sum of one evaluation's class-sweep dispatches
    (class sweep; evaluations counted by cls_root_kernel dispatches)."""
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "-d", out_dir, "-o", "run",
           "--output-format", "csv", "--", sys.executable, os.path.join(ROOT, "bench.py")] + bench_args
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                   env=dict(os.environ, TMPDIR="/tmp"), timeout=900)
    total, n = 0.0, 0
    for f in glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            if engine == "class":
                if any(k in name for k in CLASS_KERNELS):
                    total += float(r["Counter_Value"])
                    n += "cls_root_kernel" in name
            elif "sweep_kernel" in name:
                total += float(r["Counter_Value"])
                n += 1
    if not n:
        raise RuntimeError("no %s samples for the %s sweep" % (counter, engine))
    return total / n, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="fluA")
    ap.add_argument("--draws", type=int, default=None)
    ap.add_argument("--engine", choices=["pattern", "class"], default="pattern")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--scratch", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    args = ap.parse_args()
    from bench import kernel_source_hash
    draws = args.draws or (1 if args.workload == "synthetic" else 8192)
    bench_args = ["--workload", args.workload, "--draws", str(draws), "--steps", "3", "--warmup", "1",
                  "--no-cpu-baseline", "--no-sampler-latency", "--no-synthetic", "--engine", args.engine]
    tag = "%s_%s" % (args.workload, args.engine)
    fetch, nf = run_pass("FETCH_SIZE", os.path.join(args.scratch, tag + "_fetch"), bench_args, args.engine)
    write, nw = run_pass("WRITE_SIZE", os.path.join(args.scratch, tag + "_write"), bench_args, args.engine)
    traffic = (2.0 * fetch + write) * 1024.0
    rec = {}
    if os.path.exists(args.out):
        try:
            rec = json.load(open(args.out))
        except ValueError:
            rec = {}
    if rec.get("kernel_source") != kernel_source_hash():
        rec = {"kernel_source": kernel_source_hash(), "per_launch_bytes": {}, "raw": {}}
    key = "%s:%d:%s" % (args.workload, draws, args.engine)
    rec["per_launch_bytes"][key] = traffic
    rec["raw"][key] = {"FETCH_SIZE_KB": fetch, "WRITE_SIZE_KB": write, "dispatches": [nf, nw],
                       "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)"}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fp:
        json.dump(rec, fp, indent=1)
    print(json.dumps({key: rec["raw"][key], "traffic_bytes": traffic}))


if __name__ == "__main__":
    main()
