set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01d; mkdir -p $O
timeout -k 10 300 python -m pytest tests/ -q -m gpu > $O/pytest.log 2>&1; tail -15 $O/pytest.log
B="timeout -k 10 200 python bench.py --no-cpu-baseline"
S="timeout -k 10 200 python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline"
$B --single-eval > $O/fluA_auto.json 2>&1; $B --cols 1 > $O/fluA_k1.json 2>&1
$S > $O/syn_auto.json 2>&1; $S --cols 1 > $O/syn_k1.json 2>&1
for f in $O/*.json; do python -c "
import json,sys
try:
    d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value'],1), d['ms_per_step'], d['roofline']['kernel_avg_ms'], round(d['roofline']['frac'],3), d['program'], d.get('single_eval'))
except Exception as e: print('$f', 'ERR', open('$f').read()[-300:])
"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > /dev/null 2>&1; cat $O/prof/run_kernel_stats.csv | cut -c1-200
