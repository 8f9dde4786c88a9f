# Quick check: GPU parity + inference tests, then the default fluA bench line.
#   gpurun --timeout 900 -- bash tools/gpu_quick2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-q}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_class.py tests/test_gpu_resident.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --json-out $O/fluA.json > $O/fluA.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/rp -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/rp.log 2>&1 && echo ALLDONE
tail -2 $O/test.log
python -c "import json; d=json.load(open('$O/fluA.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
