# Class-sweep GPU check (run through gpurun): tests, then the synthetic bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cls}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_class.py -x -v --timeout 200 --timeout-method thread > $O/pytest_class.log 2>&1; rc=$?
tail -5 $O/pytest_class.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload synthetic --steps 20 --warmup 3 --no-cpu-baseline --json-out $O/syn.json > $O/syn.log 2>&1 && cat $O/syn.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_syn -o run --output-format csv -- python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > $O/syn_rp.log 2>&1 && \
echo ALLDONE
