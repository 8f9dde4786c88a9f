# A/B of the product library against variant builds on one box (alternating runs).
#   gpurun --timeout 900 -- bash tools/gpu_ab3.sh TAG variants/x.so [variants/y.so ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -5 $O/test.log; exit 1; }
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --json-out $O/base_$rep.json > $O/base_$rep.log 2>&1 || exit $?
  for v in "$@"; do
    n=$(basename $v .so)
    PHYLO_HIP_AB=1 PHYLO_HIP_LIB=$PWD/$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --json-out $O/${n}_$rep.json > $O/${n}_$rep.log 2>&1 || exit $?
  done
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), round(d['roofline']['kernel_avg_ms'],4))"; done
