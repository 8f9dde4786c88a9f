set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && tail -3 $O/pytest.log && \
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/fluA.json 2> $O/fluA.err && cat $O/fluA.json && \
timeout -k 10 200 python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > $O/syn.json 2> $O/syn.err && cat $O/syn.json
