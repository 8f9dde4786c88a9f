#!/usr/bin/env python
"""Collect SQ / TCC counters of the sweep kernel in separate rocprofv3 --pmc
passes (kernel-trace only) and print per-dispatch averages.  Run on the GPU
box:  python tools/pmc_sq.py [bench.py args ...]
PMC_KERNEL=name: that kernel's dispatches only; PMC_SCRIPT=tools/latency_probe.py:
profile that script (with the given args) instead of bench.py."""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU",
    "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT",
    "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS",
    "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum",
]


def main():
    bench_args = sys.argv[1:] or ["--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-synthetic"]
    out = {}
    for k, counters in enumerate(PASSES):
        d = os.path.join(ROOT, "gpurun_out", "pmc_sq", "p%d" % k)
        cmd = ["rocprofv3", "--kernel-trace", "-d", d, "-o", "run", "--output-format", "csv"]
        cmd += ["--pmc"] + counters.split()
        script = os.environ.get("PMC_SCRIPT", "bench.py")
        cmd += ["--", sys.executable, os.path.join(ROOT, script)] + bench_args
        r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=180,
                           env=dict(os.environ, TMPDIR="/tmp"))
        if r.returncode != 0:
            print("pass %d failed: %s" % (k, r.stderr.decode()[-2000:]), file=sys.stderr)
            continue
        # pattern sweep: average per sweep_kernel dispatch; class sweep: the
        # sum over one evaluation's cls_* dispatches (evaluations counted by
        # cls_root_kernel)
        cls = "class" in bench_args
        only = os.environ.get("PMC_KERNEL")  # e.g. res_rev_kernel: that kernel's dispatches only
        acc, nev = {}, {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                name = row["Kernel_Name"]
                if only:
                    if only not in name:
                        continue
                elif cls:
                    if "cls_" not in name or "epi" in name or "site" in name:
                        continue
                elif "sweep_kernel" not in name:
                    continue
                cn = row["Counter_Name"]
                acc[cn] = acc.get(cn, 0.0) + float(row["Counter_Value"])
                if only or not cls or "cls_root_kernel" in name:
                    nev[cn] = nev.get(cn, 0) + 1
        for cn, v in acc.items():
            out[cn] = v / max(nev.get(cn, 1), 1)
    print(json.dumps(out, indent=1))
    # keyed record for bench.py's roofline.compute (same kernel source only)
    if not os.environ.get("PMC_KERNEL") and not os.environ.get("PMC_SCRIPT") and "SQ_INSTS_VALU_FMA_F64" in out and "SQ_WAVE_CYCLES" in out:
        sys.path.insert(0, ROOT)
        from bench import kernel_source_hash
        wl = bench_args[bench_args.index("--workload") + 1] if "--workload" in bench_args else "fluA"
        eng = bench_args[bench_args.index("--engine") + 1] if "--engine" in bench_args else "pattern"
        path = os.path.join(ROOT, "profiles", "sq_counters.json")
        rec = {}
        if os.path.exists(path):
            try:
                rec = json.load(open(path))
            except ValueError:
                rec = {}
        if rec.get("kernel_source") != kernel_source_hash():
            rec = {"kernel_source": kernel_source_hash(), "per_launch": {}}
        rec["per_launch"]["%s:%s" % (wl, eng)] = out
        with open(path, "w") as fp:
            json.dump(rec, fp, indent=1)


if __name__ == "__main__":
    main()
