#!/bin/bash
# Round-3 profiles:  gpurun --timeout 1200 -- bash tools/gpu_r03_prof.sh TAG
# Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r03}
O=gpurun_out/prof_$TAG; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_fluA -o run --output-format csv -- python bench.py --no-cpu-baseline --no-sampler-latency --json-out $O/fluA_under_rocprof.json > $O/fluA_rp.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/rp_lat -o run --output-format csv -- python tools/latency_probe.py --draws 4 --calls 300 > $O/lat_rp.log 2>&1 && \
timeout -k 10 200 python tools/pmc_traffic.py --workload fluA --engine pattern --scratch $O/pmc > $O/pmc_fluA.log 2>&1 && \
cp profiles/pmc_traffic.json $O/pmc_traffic.json && \
timeout -k 10 400 python tools/pmc_sq.py --workload fluA --engine pattern --steps 3 --warmup 1 --no-cpu-baseline --no-sampler-latency > $O/sq_fluA.json 2> $O/sq_fluA.err && \
for n in 8; do timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_shard$n -o run --output-format csv -- python bench.py --workload synthetic --shard-of $n --steps 50 --warmup 5 --no-cpu-baseline --json-out $O/syn_shard${n}_rp.json > $O/syn_shard${n}_rp.log 2>&1 || exit $?; done && \
timeout -k 10 300 python bench.py --json-out $O/fluA.json > $O/fluA.log 2>&1 && \
cat $O/fluA.json && echo ALLDONE
