#!/bin/bash
# config 5 (full NUTS on fluA) per engine, after the -m gpu suite:
#   gpurun -- bash tools/gpu_r03_cfg5.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/cfg5_${1:-a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -4 $O/tests.log
for e in latency pattern; do
  timeout -k 10 300 python tools/run_config5.py --engine $e --out $O/$e > $O/$e.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('$O/$e/config5.json')); print('$e', d['engine'], 'wall %.2f s' % d['wall_s'], 'grads', d['gradient_evaluations'], '%.0f grads/s' % d['grads_per_s'], {k: round(v['mean'], 5) for k, v in d['summary'].items()}, all(v['mean_within_reference_ci'] for v in d['summary'].values()))"
done
