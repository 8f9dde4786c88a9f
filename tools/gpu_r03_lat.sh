#!/bin/bash
# GPU suite, then small-batch latency per engine and a short fluA bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/lat_r03; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ge 124 ] && exit $rc
for e in pattern resident; do for d in 1 4 16; do
  timeout -k 10 60 python tools/latency_probe.py --draws $d --calls 300 --engine $e >> $O/lat.jsonl 2>> $O/lat.err || exit 1
done; done
cat $O/lat.jsonl
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/rp_lat -o run --output-format csv -- python tools/latency_probe.py --draws 4 --calls 200 > $O/lat_rp.log 2>&1 && head -8 $O/rp_lat/run_kernel_stats.csv
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --json-out $O/fluA.json > $O/fluA.log 2>&1 && tail -c 1500 $O/fluA.json
