# What the driver runs at round end (through gpurun): the GPU suite, smoke(), the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-drv}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.log && tail -c 400 $O/bench.json && echo ALLDONE
