#!/bin/bash
# Round-3 profiles:  gpurun --timeout 1200 -- bash tools/gpu_r03_prof.sh TAG
# Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r03}
O=gpurun_out/prof_$TAG; mkdir -p $O
timeout -k 10 200 python tools/pmc_traffic.py --workload fluA --engine pattern --scratch $O/pmc > $O/pmc_fluA.log 2>&1 && \
timeout -k 10 300 python tools/pmc_traffic.py --workload synthetic --engine class --scratch $O/pmc > $O/pmc_syn.log 2>&1 && \
timeout -k 10 200 python tools/pmc_traffic.py --workload HCV --engine pattern --scratch $O/pmc > $O/pmc_HCV.log 2>&1 && \
timeout -k 10 200 python tools/pmc_traffic.py --workload DS1 --engine pattern --scratch $O/pmc > $O/pmc_DS1.log 2>&1 && \
timeout -k 10 400 python tools/pmc_sq.py --workload fluA --engine pattern --steps 3 --warmup 1 --no-cpu-baseline --no-sampler-latency > $O/sq_fluA.json 2> $O/sq_fluA.err && \
timeout -k 10 400 python tools/pmc_sq.py --workload HCV --engine pattern --steps 3 --warmup 1 --no-cpu-baseline --no-sampler-latency > $O/sq_HCV.json 2> $O/sq_HCV.err && \
timeout -k 10 400 python tools/pmc_sq.py --workload DS1 --engine pattern --steps 3 --warmup 1 --no-cpu-baseline --no-sampler-latency > $O/sq_DS1.json 2> $O/sq_DS1.err && \
timeout -k 10 600 python tools/pmc_sq.py --workload synthetic --engine class --steps 3 --warmup 1 --no-cpu-baseline --no-sampler-latency > $O/sq_syn.json 2> $O/sq_syn.err && \
cp profiles/pmc_traffic.json profiles/sq_counters.json $O/ && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_fluA -o run --output-format csv -- python bench.py --no-cpu-baseline --no-sampler-latency --json-out $O/fluA_under_rocprof.json > $O/fluA_rp.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/rp_lat -o run --output-format csv -- python tools/latency_probe.py --draws 4 --calls 300 > $O/lat_rp.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_syn -o run --output-format csv -- python bench.py --workload synthetic --steps 20 --warmup 3 --no-cpu-baseline --json-out $O/syn_under_rocprof.json > $O/syn_rp.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_shard8 -o run --output-format csv -- python bench.py --workload synthetic --shard-of 8 --steps 50 --warmup 5 --no-cpu-baseline --json-out $O/syn_shard8_rp.json > $O/syn_shard8_rp.log 2>&1 && \
echo PROFDONE
