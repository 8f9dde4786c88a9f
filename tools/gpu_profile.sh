# Refresh the committed profiles for the current kernel source (run through gpurun):
#   gpurun --timeout 1100 -- bash tools/gpu_profile.sh r01
# Every GPU step has its own time limit and the steps are chained with &&.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out/prof_$TAG; mkdir -p $O
timeout -k 10 200 python tools/pmc_traffic.py --workload fluA --scratch $O/pmc > $O/pmc_fluA.log 2>&1 && \
timeout -k 10 300 python tools/pmc_traffic.py --workload synthetic --scratch $O/pmc > $O/pmc_syn.log 2>&1 && \
cp profiles/pmc_traffic.json $O/pmc_traffic.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_fluA -o run --output-format csv -- python bench.py --no-cpu-baseline > $O/fluA_under_rocprof.json 2> $O/fluA_under_rocprof.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_syn -o run --output-format csv -- python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > $O/syn_under_rocprof.json 2> $O/syn_under_rocprof.err && \
timeout -k 10 300 python bench.py --single-eval > $O/fluA.json 2> $O/fluA.err && \
timeout -k 10 300 python bench.py --workload synthetic --steps 20 --warmup 3 > $O/syn.json 2> $O/syn.err && \
cat $O/fluA.json $O/syn.json && find $O -name '*kernel_stats.csv' -o -name '*counter_collection.csv'
