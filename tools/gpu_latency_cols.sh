set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lat; mkdir -p $O
timeout -k 10 200 python bench.py --single-eval --no-cpu-baseline --steps 20 --warmup 3 --json-out $O/k2.json > $O/k2.log 2>&1 && \
timeout -k 10 200 python bench.py --single-eval --cols 1 --no-cpu-baseline --steps 20 --warmup 3 --json-out $O/k1.json > $O/k1.log 2>&1 && \
timeout -k 10 200 python bench.py --workload HCV --single-eval --no-cpu-baseline --steps 20 --warmup 3 --json-out $O/h2.json > $O/h2.log 2>&1 && \
timeout -k 10 200 python bench.py --workload HCV --single-eval --cols 1 --no-cpu-baseline --steps 20 --warmup 3 --json-out $O/h1.json > $O/h1.log 2>&1
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['single_eval'], round(d['value']))"; done
