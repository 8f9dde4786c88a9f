# fluA / HCV bench per library variant from variants/ (run through gpurun): $1 = tag, then variant names
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-var}; mkdir -p $O; shift
for v in "$@"; do
  for w in fluA HCV; do
    PHYLO_HIP_LIB=variants/libphylo_hip_$v.so timeout -k 10 300 python bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline > $O/${w}_$v.json 2> $O/${w}_$v.log || exit 1
    python -c "import json; r=json.loads(open('$O/${w}_$v.json').read().strip().splitlines()[-1]); print('$w $v', round(r['roofline']['kernel_avg_ms'],4), round(r['value']), r['program']['recomputed'])"
  done
done
echo ALLDONE
