#!/bin/bash
# site sharding of fluA (one GPU evaluates the first of N pattern
# shards for all 8192 draws; no collective) beside the replica headline.
#   gpurun --timeout 600 -- bash tools/gpu_r03_fluA_shards.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-fluA_shards}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-sampler-latency --json-out $O/fluA.json > $O/fluA.log 2>&1 || exit $?
for n in 2 4; do
  timeout -k 10 200 python bench.py --shard-of $n --steps 50 --warmup 5 --no-cpu-baseline --no-sampler-latency --json-out $O/fluA_shard$n.json > $O/fluA_shard$n.log 2>&1 || exit $?
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), d['ms_per_step'], d['config']['patterns_per_rank'], d['program']['nblocks'])"; done
