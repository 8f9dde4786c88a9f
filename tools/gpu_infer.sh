# Inference checks on the GPU (run through gpurun): the inference tests, config 5 summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-inf}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_class.py tests/test_gpu_inference.py -x -v --timeout 400 --timeout-method thread > $O/pytest_inf.log 2>&1; rc=$?
tail -12 $O/pytest_inf.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/run_config5.py --out $O/config5 > $O/config5.log 2>&1 && tail -1 $O/config5.log && echo ALLDONE
