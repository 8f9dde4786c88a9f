#!/bin/bash
# A/B of the small path's direct host I/O (PHY_DIRECT_IN / PHY_DIRECT_OUT; a source variant,
# measured and not kept -- DESIGN.md 9, profiles/r03_direct_io_ab.jsonl):
# 4-draw calls, each setting twice, alternating; then the parity tests with both on.
set -o pipefail
O=gpurun_out/dio
mkdir -p $O
: > $O/lat.jsonl
for rep in 1 2; do
  for f in "0 0" "1 0" "0 1" "1 1"; do
    set -- $f
    for w in "fluA resident" "HCV resident" "DS1 pattern" "fluA pattern"; do
      set -- $f $w
      PHY_DIRECT_IN=$1 PHY_DIRECT_OUT=$2 timeout -k 10 60 python tools/latency_probe.py --draws 4 --workload $3 --engine $4 \
        | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); d['din']=$1; d['dout']=$2; print(json.dumps(d))" >> $O/lat.jsonl || exit 1
    done
  done
done
PHY_DIRECT_IN=1 PHY_DIRECT_OUT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_resident.py tests/test_gpu_inference.py tests/test_gpu_00_configs.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
exit $rc
