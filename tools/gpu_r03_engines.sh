#!/bin/bash
# Pattern vs resident engine on the sampler's path: small-call latency
# (fluA / HCV, 1 / 4 / 16 draws, alternating) and config 5 (full NUTS on fluA)
# on each engine; the new bitwise host/device eigensystem test first.
#   gpurun --timeout 900 -- bash tools/gpu_r03_engines.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-engines}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "eigensystems or submit_wait or production" --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
for rep in 1 2; do
  for eng in pattern resident; do
    for w in fluA HCV; do for d in 1 4 16; do
      timeout -k 10 60 python tools/latency_probe.py --workload $w --draws $d --calls 300 --engine $eng >> $O/lat_$eng.jsonl 2>> $O/err.log || exit $?
    done; done
  done
done
for eng in pattern resident; do
  timeout -k 10 200 python tools/run_config5.py --engine $eng --out $O/config5_$eng > $O/config5_$eng.log 2>&1 || exit $?
  tail -3 $O/config5_$eng.log
done
for f in $O/*.jsonl; do echo "$f"; cat $f; done
