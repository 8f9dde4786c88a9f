# Interleaved A/B (A B A B ...) of engine builds on the fluA bench, for
# differences near the run-to-run noise:  gpurun -- bash tools/gpu_ab2.sh TAG ROUNDS LIB...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
for r in $(seq 1 $R); do
  for L in "$@"; do
    n=$(basename $L .so)
    PHYLO_HIP_LIB=$PWD/$L timeout -k 10 240 python bench.py --steps 100 --warmup 10 --no-cpu-baseline ${BENCH_ARGS} > $O/${n}_$r.json 2> $O/${n}_$r.err || exit $?
    echo "$n $r $(python -c "import json;d=json.load(open('$O/${n}_$r.json'));print(round(d['value']), round(d['roofline']['kernel_avg_ms'],4))")"
  done
done
