set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_inference.py -x -v --timeout 500 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -15 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u tools/run_config5.py --chains 4 --out $O/config5 > $O/config5.log 2>&1; rc=$?; tail -5 $O/config5.log; exit $rc
