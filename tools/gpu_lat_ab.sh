#!/bin/bash
# Sampler-call latency A/B: the product library against variant builds,
# alternating on one box.  Outputs under gpurun_out/TAG/.
#   gpurun --timeout 600 -- bash tools/gpu_lat_ab.sh TAG "fluA HCV" 4 variants/x.so [variants/y.so ...]
set -eo pipefail
export TMPDIR=/tmp
TAG=$1; WLS=$2; D=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  for w in $WLS; do
    timeout -k 10 120 python tools/latency_probe.py --workload $w --draws $D --engine pattern > $O/base_${w}_$rep.log 2>&1
    echo "base $w rep$rep $(tail -1 $O/base_${w}_$rep.log)"
    for v in "$@"; do
      n=$(basename $v .so)
      PHYLO_HIP_AB=1 PHYLO_HIP_LIB=$PWD/$v timeout -k 10 120 python tools/latency_probe.py --workload $w --draws $D \
        --engine pattern > $O/${n}_${w}_$rep.log 2>&1
      echo "$n $w rep$rep $(tail -1 $O/${n}_${w}_$rep.log)"
    done
  done
done
