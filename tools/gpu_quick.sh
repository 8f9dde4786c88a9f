# Quick GPU iteration (run through gpurun): GPU tests, then the fluA and
# synthetic bench lines.
# $1 = output tag, $2 = extra pytest -k filter.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-quick}; mkdir -p $O
K=${2:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/fluA.json 2> $O/fluA.log && tail -c 700 $O/fluA.json &&
timeout -k 10 300 python bench.py --workload synthetic --steps 50 --warmup 5 --no-cpu-baseline > $O/syn.json 2> $O/syn.log && tail -c 300 $O/syn.json && echo ALLDONE
