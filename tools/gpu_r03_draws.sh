#!/bin/bash
# Latency per call vs draws per call (fluA / HCV; 4..128 draws) per
# environment setting, alternating twice.
#   gpurun --timeout 900 -- bash tools/gpu_r03_draws.sh TAG "PHY_LAT_WPS=1" "PHY_LAT_WPS=2"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  for e in "$@"; do
    n=$(echo "$e" | tr ' =' '__')
    for w in fluA HCV; do for d in 32 64 100 128; do
      env $e timeout -k 10 60 python tools/latency_probe.py --workload $w --draws $d --calls 200 --engine pattern >> $O/lat_$n.jsonl 2>> $O/err.log || exit $?
    done; done
  done
done
for f in $O/*.jsonl; do echo "$f"; python -c "
import json,sys
for l in open('$f'): d=json.loads(l); print(d['workload'], d['draws'], round(d['us_per_call'],1))"; done
