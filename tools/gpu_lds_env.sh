# LDS plan experiments through environment variables (no rebuild).
#   gpurun --timeout 600 -- bash tools/gpu_lds_env.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ldsenv}; mkdir -p $O
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --json-out $O/base.json > $O/base.log 2>&1 || exit $?
PHY_LDS_BUDGET=163840 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --json-out $O/one.json > $O/one.log 2>&1 || exit $?
PHY_LDS_BUDGET=163840 PHY_DEEP=2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --json-out $O/one_g.json > $O/one_g.log 2>&1 || exit $?
PHY_DEEP=2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --json-out $O/deepg.json > $O/deepg.log 2>&1 || exit $?
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); p=d['program']; print('$f', round(d['value']), round(d['roofline']['kernel_avg_ms'],3), p['n_chunks'], p['matrices_per_chunk'], p['lds_bytes'], p['deep_lds_entries'], p['recomputed'])"; done
