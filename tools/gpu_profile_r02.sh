# Round-2 profiles (run through gpurun):  gpurun --timeout 1200 -- bash tools/gpu_profile_r02.sh TAG
# Every GPU step has its own time limit and the steps are chained with &&.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
O=gpurun_out/prof_$TAG; mkdir -p $O
timeout -k 10 200 python tools/pmc_traffic.py --workload fluA --engine pattern --scratch $O/pmc > $O/pmc_fluA.log 2>&1 && \
timeout -k 10 300 python tools/pmc_traffic.py --workload synthetic --engine class --scratch $O/pmc > $O/pmc_syn.log 2>&1 && \
timeout -k 10 200 python tools/pmc_traffic.py --workload HCV --engine pattern --scratch $O/pmc > $O/pmc_HCV.log 2>&1 && \
timeout -k 10 200 python tools/pmc_traffic.py --workload DS1 --engine pattern --scratch $O/pmc > $O/pmc_DS1.log 2>&1 && \
cp profiles/pmc_traffic.json $O/pmc_traffic.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_fluA -o run --output-format csv -- python bench.py --no-cpu-baseline --json-out $O/fluA_under_rocprof.json > $O/fluA_rp.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_syn -o run --output-format csv -- python bench.py --workload synthetic --steps 20 --warmup 3 --no-cpu-baseline --json-out $O/syn_under_rocprof.json > $O/syn_rp.log 2>&1 && \
timeout -k 10 300 python bench.py --single-eval --json-out $O/fluA.json > $O/fluA.log 2>&1 && \
timeout -k 10 300 python bench.py --workload synthetic --steps 50 --warmup 5 --json-out $O/syn.json > $O/syn.log 2>&1 && \
timeout -k 10 300 python bench.py --workload synthetic --engine pattern --steps 20 --warmup 3 --no-cpu-baseline --json-out $O/syn_pattern.json > $O/syn_pattern.log 2>&1 && \
timeout -k 10 300 python bench.py --workload HCV --json-out $O/HCV.json > $O/HCV.log 2>&1 && \
timeout -k 10 300 python bench.py --workload DS1 --json-out $O/DS1.json > $O/DS1.log 2>&1 && \
for n in 2 4 8; do timeout -k 10 300 python bench.py --workload synthetic --shard-of $n --steps 50 --warmup 5 --no-cpu-baseline --json-out $O/syn_shard$n.json > $O/syn_shard$n.log 2>&1 || exit $?; done && \
timeout -k 10 400 python tools/pmc_sq.py --workload synthetic --engine class --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_syn_class.json 2> $O/sq_syn_class.err && \
timeout -k 10 400 python tools/pmc_sq.py --workload fluA --engine pattern --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_fluA.json 2> $O/sq_fluA.err && \
cat $O/fluA.json $O/syn.json && echo ALLDONE
