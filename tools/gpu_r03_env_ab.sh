#!/bin/bash
# Same-box A/B of environment settings of the product library:
# parity tests (default env), then fluA 4-draw latency and the fluA bench
# per setting, alternating twice.
#   gpurun --timeout 900 -- bash tools/gpu_r03_env_ab.sh TAG "PHY_GL=0" "PHY_GL=1" ...
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
    env $e timeout -k 10 60 python tools/latency_probe.py --draws 4 --calls 300 >> $O/lat_$n.jsonl 2>> $O/err.log || exit $?
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-sampler-latency --steps 50 --warmup 5 --json-out $O/${n}_$rep.json > $O/${n}_$rep.log 2>&1 || exit $?
  done
done
for f in $O/*.jsonl; do echo "$f"; cat $f; done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); p=d['program']; print('$f', round(d['value']), round(d['roofline']['kernel_avg_ms'],4), p['n_chunks'], p['matrices_per_chunk'], p['lds_bytes'])"; done
