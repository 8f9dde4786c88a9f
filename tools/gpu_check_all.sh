# Full GPU check (run through gpurun):  gpurun --timeout 1200 -- bash tools/gpu_check_all.sh TAG
# pytest -m gpu, the fluA / synthetic bench lines, then the SQ counter passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-chk}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
tail -3 $O/pytest_gpu.log && \
timeout -k 10 300 python bench.py --json-out $O/fluA.json > $O/fluA.log 2>&1 && cat $O/fluA.json && \
timeout -k 10 300 python bench.py --workload synthetic --steps 20 --warmup 3 --json-out $O/syn.json > $O/syn.log 2>&1 && cat $O/syn.json && \
timeout -k 10 400 python tools/pmc_sq.py --steps 20 --warmup 2 --no-cpu-baseline > $O/sq_fluA.json 2> $O/sq_fluA.err && \
timeout -k 10 400 python tools/pmc_sq.py --workload synthetic --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_syn.json 2> $O/sq_syn.err && \
echo ALLDONE
