set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r01
timeout -k 10 300 python -m pytest tests/ -q -m gpu 2>&1 | grep -E "^E |passed|failed|^FAILED" | head -20
timeout -k 10 300 python tools/pmc_traffic.py --workload fluA
timeout -k 10 600 python tools/pmc_traffic.py --workload synthetic
cp profiles/pmc_traffic.json gpurun_out/r01/pmc_traffic.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r01/prof_fluA -o run --output-format csv -- python bench.py > gpurun_out/r01/bench_under_rocprof.json 2> gpurun_out/r01/bench_under_rocprof.err
timeout -k 10 300 python bench.py --single-eval > gpurun_out/r01/bench.json 2> gpurun_out/r01/bench.err
cat gpurun_out/r01/bench.json
timeout -k 10 300 python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r01/bench_synth.json 2> gpurun_out/r01/bench_synth.err
cat gpurun_out/r01/bench_synth.json
rocprofv3 -L > gpurun_out/r01/counters.txt 2>&1 || true
