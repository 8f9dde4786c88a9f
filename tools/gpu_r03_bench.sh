#!/bin/bash
# Round-3 benches:  gpurun --timeout 1200 -- bash tools/gpu_r03_bench.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r03}
O=gpurun_out/bench_$TAG; mkdir -p $O
timeout -k 10 300 python bench.py --json-out $O/fluA.json > $O/fluA.log 2>&1 && \
timeout -k 10 300 python bench.py --workload HCV --json-out $O/HCV.json > $O/HCV.log 2>&1 && \
timeout -k 10 300 python bench.py --workload DS1 --json-out $O/DS1.json > $O/DS1.log 2>&1 && \
timeout -k 10 300 python bench.py --workload synthetic --steps 50 --warmup 5 --json-out $O/syn.json > $O/syn.log 2>&1 && \
for n in 2 4 8; do timeout -k 10 300 python bench.py --workload synthetic --shard-of $n --steps 50 --warmup 5 --no-cpu-baseline --json-out $O/syn_shard$n.json > $O/syn_shard$n.log 2>&1 || exit $?; done && \
timeout -k 10 300 python tools/run_config5.py --out $O/config5 > $O/config5.log 2>&1 && \
cat $O/fluA.json && echo ALLDONE
