# GPU check: the whole -m gpu suite, then the synthetic bench line (class
# sweep, with cpu_baseline) and its rocprofv3 kernel stats.
#   gpurun --timeout 1200 -- bash tools/gpu_check_syn.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-chk}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload synthetic --steps 20 --warmup 3 --json-out $O/syn.json > $O/syn.log 2>&1 && cat $O/syn.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_syn -o run --output-format csv -- python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > $O/syn_rp.log 2>&1 && \
echo ALLDONE
