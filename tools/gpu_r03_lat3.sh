#!/bin/bash
# Parity tests, then small-call latency per environment setting (fluA and
# HCV, 1/4/16 draws) and a kernel trace of 4-draw fluA calls.
#   gpurun --timeout 900 -- bash tools/gpu_r03_lat3.sh TAG "PHY_KLAT=0" "PHY_KLAT=1"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_00_configs.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
for rep in 1 2; do
  for e in "$@"; do
    n=$(echo "$e" | tr ' =' '__')
    for w in fluA HCV; do for d in 1 4 16; do
      env $e timeout -k 10 60 python tools/latency_probe.py --workload $w --draws $d --calls 300 >> $O/lat_$n.jsonl 2>> $O/err.log || exit $?
    done; done
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/rp_lat -o run --output-format csv -- python tools/latency_probe.py --draws 4 --calls 300 > $O/lat_rp.log 2>&1 || exit $?
for f in $O/*.jsonl; do echo "$f"; cat $f; done
cut -d, -f1-4 $O/rp_lat/run_kernel_stats.csv
