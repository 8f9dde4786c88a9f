# A/B of sweep-kernel builds on both bench workloads.
#   gpurun -- bash tools/gpu_ab.sh TAG LIB1 [LIB2 ...]   (LIB "cur" = in-tree build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = cur ]; then unset PHYLO_HIP_LIB; else export PHYLO_HIP_LIB=$PWD/$L; fi
  timeout -k 10 240 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/fluA_$n.json 2> $O/fluA_$n.err || exit $?
  echo "$n fluA $(python -c "import json;d=json.load(open('$O/fluA_$n.json'));print(d['value'],d['roofline']['frac'])")"
  [ -n "$FLUA_ONLY" ] && continue
  timeout -k 10 300 python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > $O/syn_$n.json 2> $O/syn_$n.err || exit $?
  echo "$n syn $(python -c "import json;d=json.load(open('$O/syn_$n.json'));print(d['value'],d['roofline']['frac'])")"
done
