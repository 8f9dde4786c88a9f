# Both engines on the batched workloads (run through gpurun):
#   gpurun -- bash tools/gpu_engines.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-eng}; mkdir -p $O
for w in fluA HCV DS1; do
  for e in pattern class; do
    timeout -k 10 300 python bench.py --workload $w --engine $e --steps 50 --warmup 5 --no-cpu-baseline --json-out $O/${w}_$e.json > $O/${w}_$e.log 2>&1 || exit $?
    echo "$w $e $(python -c "import json;d=json.load(open('$O/${w}_$e.json'));print(round(d['value']), round(d['roofline']['kernel_avg_ms'],3), round(d['ms_per_step'],3))")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_fluA_class -o run --output-format csv -- python bench.py --engine class --steps 10 --warmup 2 --no-cpu-baseline > $O/fluA_class_rp.log 2>&1 && echo ALLDONE
