#!/bin/bash
# Small-call latency by plan (columns per lane, LDS share) and eigensystem
# placement:  gpurun -- bash tools/gpu_lat_k.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/latk_${1:-a}; mkdir -p $O
run() {  # name, env, probe args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/rp_$name -o run --output-format csv -- \
    python tools/latency_probe.py --draws 4 --calls 300 "$@" > $O/$name.log 2>&1 || return $?
  echo "$name $(grep us_per_call $O/$name.log)"
}
run base "PHY_HOST_EIG=1" && run deveig "PHY_HOST_EIG=0" && run k1 "PHY_HOST_EIG=1" --cols 1 && \
run k1lds "PHY_HOST_EIG=1" --cols 1 --lds-budget 163840 && run k2lds "PHY_HOST_EIG=1" --cols 2 --lds-budget 163840 && \
run res "PHY_HOST_EIG=1" --engine resident && \
for d in 1 16; do
  timeout -k 10 120 python tools/latency_probe.py --draws $d --calls 300 || exit $?
  timeout -k 10 120 python tools/latency_probe.py --draws $d --calls 300 --cols 1 || exit $?
done
