set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x 2>&1 | grep -E "^E |passed|failed|^FAILED" | head -20
timeout -k 10 100 python stamp_probe.py
for d in 1 2048; do
  for L in 163840 81920 54000; do
    timeout -k 10 120 python bench.py --steps 30 --warmup 3 --draws $d --lds-budget $L --no-cpu-baseline > gpurun_out/b_${d}_${L}.json 2> gpurun_out/b_${d}_${L}.err || { echo "FAIL $d $L"; tail -5 gpurun_out/b_${d}_${L}.err; exit 1; }
    python -c "import json;r=json.load(open('gpurun_out/b_${d}_${L}.json'));print($d,$L,'%.0f evals/s'%r['value'],'ms/step %.3f'%r['ms_per_step'],'kern %.3f ms'%r['roofline']['kernel_avg_ms'],'frac %.3f'%r['roofline']['frac'], r['program'])"
  done
done
