# Compare prebuilt diagnostic variants of the engine (build/*.so) on the bench
# workloads; optional SQ counter passes.  Run through gpurun:
#   gpurun -- bash tools/gpu_variants.sh TAG "variant1 variant2 ..." [sq]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-var}; VARS=${2:-}; SQ=${3:-}
O=gpurun_out/$TAG; mkdir -p $O
B="timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10"
S="timeout -k 10 120 python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline"
summ() { python -c "
import json,sys
d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', round(d['value'],1), round(d['roofline']['kernel_avg_ms'],4), round(d['roofline']['frac'],3), d['program'])
"; }
$B > $O/fluA_base.json 2> $O/fluA_base.err && summ $O/fluA_base.json && \
$S > $O/syn_base.json 2> $O/syn_base.err && summ $O/syn_base.json || exit 1
for v in $VARS; do
  lib=$PWD/build/${v%%@*}.so; extra=""; case $v in *@*) extra=$(echo ${v#*@} | tr ',' ' ');; esac
  PHYLO_HIP_LIB=$lib $B $extra > $O/fluA_$v.json 2> $O/fluA_$v.err && summ $O/fluA_$v.json && \
  PHYLO_HIP_LIB=$lib $S $extra > $O/syn_$v.json 2> $O/syn_$v.err && summ $O/syn_$v.json || exit 1
done
if [ -n "$SQ" ]; then
  timeout -k 10 400 python tools/pmc_sq.py --workload synthetic --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_syn.json 2> $O/sq_syn.err && cat $O/sq_syn.json
fi
