set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/icache; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH -d $O/p0 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/b.err
python - <<'PY'
import csv, glob
acc={}
for f in glob.glob("gpurun_out/icache/p0/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sweep_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k,v in acc.items(): print(k, sum(v)/len(v))
PY
