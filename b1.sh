set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x 2>&1 | tail -2
for d in 1 2048; do
  for L in 0 80000; do
    timeout -k 10 120 python bench.py --steps 30 --warmup 3 --draws $d --lds-budget $L --no-cpu-baseline > gpurun_out/b_${d}_${L}.json 2> gpurun_out/b_${d}_${L}.err || { echo "FAIL $d $L"; tail -5 gpurun_out/b_${d}_${L}.err; exit 1; }
    python -c "import json;r=json.load(open('gpurun_out/b_${d}_${L}.json'));print($d,$L,'%.0f evals/s'%r['value'],'ms/step %.3f'%r['ms_per_step'],'kern %.3f ms'%r['roofline']['kernel_avg_ms'],'frac %.3f'%r['roofline']['frac'])"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 30 --warmup 3 --draws 1 --no-cpu-baseline > /dev/null 2>&1
find gpurun_out/prof1 -name "*stats*" | head
cat $(find gpurun_out/prof1 -name "*kernel_stats.csv" | head -1) | cut -c1-250
