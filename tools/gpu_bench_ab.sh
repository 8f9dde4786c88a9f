#!/bin/bash
# bench.py A/B of the product library against variant builds, alternating,
# two rounds, with the given bench arguments.  Outputs under gpurun_out/TAG/.
#   gpurun --timeout 900 -- bash tools/gpu_bench_ab.sh TAG "--workload synthetic --steps 30" variants/x.so ...
set -eo pipefail
export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline --json-out $O/base_$rep.json > $O/base_$rep.log 2>&1
  python -c "import json;d=json.load(open('$O/base_$rep.json'));print('base rep$rep', d['value'], d['ms_per_step'])"
  for v in "$@"; do
    n=$(basename $v .so)
    PHYLO_HIP_AB=1 PHYLO_HIP_LIB=$PWD/$v timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline \
      --json-out $O/${n}_$rep.json > $O/${n}_$rep.log 2>&1
    python -c "import json;d=json.load(open('$O/${n}_$rep.json'));print('$n rep$rep', d['value'], d['ms_per_step'])"
  done
done
