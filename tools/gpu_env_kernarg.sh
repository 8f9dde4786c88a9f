# Launch-latency environment check: HIP_FORCE_DEV_KERNARG on the small-kernel-bound cases.
#   gpurun --timeout 600 -- bash tools/gpu_env_kernarg.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-kernarg}; mkdir -p $O
for v in 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py --workload synthetic --shard-of 8 --steps 50 --warmup 5 --no-cpu-baseline --json-out $O/sh8_$v.json > $O/sh8_$v.log 2>&1 || exit $?
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py --workload synthetic --steps 30 --warmup 5 --no-cpu-baseline --json-out $O/syn_$v.json > $O/syn_$v.log 2>&1 || exit $?
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python tools/latency_probe.py --draws 4 --engine resident >> $O/lat.jsonl 2>> $O/lat.err || exit $?
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), round(d['ms_per_step'],4))"; done
cat $O/lat.jsonl
