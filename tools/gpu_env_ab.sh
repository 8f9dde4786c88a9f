# Interleaved A/B of environment settings on the in-tree build (fluA bench):
#   gpurun -- bash tools/gpu_env_ab.sh TAG ROUNDS "ENV1" "ENV2" ...   (ENV "" = defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
for r in $(seq 1 $R); do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 240 python bench.py --steps 100 --warmup 10 --no-cpu-baseline ${BENCH_ARGS} > $O/e${i}_$r.json 2> $O/e${i}_$r.err || exit $?
    echo "[$E] $r $(python -c "import json;d=json.load(open('$O/e${i}_$r.json'));print(round(d['value'],1), round(d['roofline']['kernel_avg_ms'],4), d['program'].get('recomputed'))")"
  done
done
