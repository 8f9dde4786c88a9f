# fluA throughput vs draws per launch (alternating).
#   gpurun --timeout 600 -- bash tools/gpu_draws.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-draws}; mkdir -p $O
for rep in 1 2; do for n in 8192 16384 32768; do
  timeout -k 10 200 python bench.py --draws $n --steps $((1638400 / n)) --warmup 5 --no-cpu-baseline --json-out $O/d${n}_$rep.json > $O/d${n}_$rep.log 2>&1 || exit $?
done; done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), round(d['roofline']['kernel_avg_ms'],3), round(d['ms_per_step'],3))"; done
