#!/bin/bash
# Round 3's committed evidence at one kernel source: the whole -m gpu suite,
# then the profiles (gpu_r03_prof.sh) and the bench lines (gpu_r03_bench.sh).
#   gpurun --timeout 1200 -- bash tools/gpu_r03_final.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r03final}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest.log 2>&1 || { tail -30 gpurun_out/$TAG/gputest.log; exit 1; }
tail -3 gpurun_out/$TAG/gputest.log
bash tools/gpu_r03_prof.sh $TAG && bash tools/gpu_r03_bench.sh $TAG
