#!/bin/bash
# round 3: GPU suite, then a short fluA bench (sampler latency included).
# A failing test does not stop the bench; a crash / timeout (exit >= 124) does.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_t.log 2>&1
rc=$?
tail -25 gpurun_out/r03_t.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03_b.log 2>&1 || { tail -20 gpurun_out/r03_b.log; exit 1; }
tail -c 3000 gpurun_out/r03_b.log
