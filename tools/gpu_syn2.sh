# Synthetic (class sweep) check: class GPU tests, then the synthetic bench line and a kernel trace.
#   gpurun --timeout 900 -- bash tools/gpu_syn2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-syn}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_class.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 && \
timeout -k 10 300 python bench.py --workload synthetic --steps 50 --warmup 5 --no-cpu-baseline --json-out $O/syn.json > $O/syn.log 2>&1 && \
timeout -k 10 300 python bench.py --workload synthetic --shard-of 8 --steps 50 --warmup 5 --no-cpu-baseline --json-out $O/syn8.json > $O/syn8.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp -o run --output-format csv -- python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > $O/rp.log 2>&1 && echo ALLDONE
tail -2 $O/test.log
for f in $O/syn.json $O/syn8.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"; done
