#!/bin/bash
# Where a small call's sweep time goes: 4-draw fluA calls (latency_probe.py)
# with the product library and diagnostic ablation builds (PHY_ABLATE bits,
# results wrong by construction, only timed), alternating twice.
#   gpurun --timeout 600 -- bash tools/gpu_lat_abl.sh TAG variants/abl2.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  for d in 4 64; do
    timeout -k 10 60 python tools/latency_probe.py --draws $d --calls 300 >> $O/base.jsonl 2>> $O/err.log || exit $?
    for v in "$@"; do
      n=$(basename $v .so)
      PHYLO_HIP_LIB=$PWD/$v timeout -k 10 60 python tools/latency_probe.py --draws $d --calls 300 >> $O/$n.jsonl 2>> $O/err.log || exit $?
    done
  done
done
for f in $O/*.jsonl; do echo "$f"; cat $f; done
