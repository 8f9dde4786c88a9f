set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu 2>&1 | grep -E "^E |passed|failed|^FAILED" | head -20
for L in 81920 163840; do
timeout -k 10 300 python bench.py --workload synthetic --steps 10 --warmup 2 --lds-budget $L --no-cpu-baseline > gpurun_out/s_$L.json 2> gpurun_out/s_$L.err || { echo FAIL; tail -5 gpurun_out/s_$L.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/s_$L.json'));print('synth',$L,'%.2f evals/s'%r['value'],'ms/step %.3f'%r['ms_per_step'],'kern %.3f ms'%r['roofline']['kernel_avg_ms'],'frac %.3f'%r['roofline']['frac'], r['config']['patterns'], r['program'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s -o run --output-format csv -- python bench.py --workload synthetic --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2>&1
cat gpurun_out/prof_s/run_kernel_stats.csv | cut -c1-200
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_s1 -o run --output-format csv -- python bench.py --workload synthetic --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_s2 -o run --output-format csv -- python bench.py --workload synthetic --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>&1
ls gpurun_out/pmc_s1 gpurun_out/pmc_s2
