#!/bin/bash
# finalize_kernel time per diagnostic build (results wrong by construction)
# in 4-draw fluA calls, from rocprofv3 kernel stats.
#   gpurun --timeout 600 -- bash tools/gpu_fin_abl.sh TAG variants/x.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/rp_base -o run --output-format csv -- python tools/latency_probe.py --draws 4 --calls 200 > $O/base.log 2>&1 || exit $?
for v in "$@"; do
  n=$(basename $v .so)
  PHYLO_HIP_LIB=$PWD/$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/rp_$n -o run --output-format csv -- python tools/latency_probe.py --draws 4 --calls 200 > $O/$n.log 2>&1 || exit $?
done
for d in $O/rp_*; do echo "$d"; grep -h finalize $d/run_kernel_stats.csv | cut -d, -f1-4; done
