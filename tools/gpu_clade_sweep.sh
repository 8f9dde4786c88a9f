# Synthetic class-sweep step time vs fused clade levels (run through gpurun); $1 = tag
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-clade}; mkdir -p $O
for sh in 1 8; do
  for c in 0 2 3 4 5; do
    PHY_CLADE=$c timeout -k 10 200 python bench.py --workload synthetic --shard-of $sh --steps 30 --warmup 3 --no-cpu-baseline > $O/s${sh}_c$c.json 2> $O/s${sh}_c$c.log || exit 1
    python -c "import json; r=json.loads(open('$O/s${sh}_c$c.json').read().strip().splitlines()[-1]); print('shard $sh clade $c', round(r['ms_per_step'],4), round(r['roofline']['kernel_avg_ms'],4), r['program'].get('class_clade_max'))"
  done
done
echo ALLDONE
