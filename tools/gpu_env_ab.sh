#!/bin/bash
# bench.py A/B over environment settings of the product library (alternating,
# two rounds):  gpurun -- bash tools/gpu_env_ab.sh TAG "BENCH ARGS" "ENV1" "ENV2" ...
# ("-" = no extra environment).  Outputs under gpurun_out/TAG/.
set -eo pipefail
export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline --no-sampler-latency \
      --json-out $O/v${i}_$rep.json > $O/v${i}_$rep.log 2>&1
    python -c "import json;d=json.load(open('$O/v${i}_$rep.json'));print('[$e] rep$rep', d['value'], d['ms_per_step'])"
  done
done
