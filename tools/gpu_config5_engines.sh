# Config 5 (full NUTS on fluA) with the automatic engine and with the resident class sweep.
#   gpurun --timeout 600 -- bash tools/gpu_config5_engines.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-c5e}; mkdir -p $O/auto $O/res
timeout -k 10 200 python tools/run_config5.py --out $O/auto > $O/auto.log 2>&1 && \
PHY_ENGINE=3 timeout -k 10 200 python tools/run_config5.py --out $O/res > $O/res.log 2>&1 && echo ALLDONE
for d in auto res; do python -c "import json; r=json.load(open('$O/$d/config5.json')); print('$d', round(r['wall_s'],2), r['gradient_evaluations'], {k:(round(v['mean'],4), v['mean_within_reference_ci']) for k,v in r['summary'].items()})"; done
