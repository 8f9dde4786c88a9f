# Sweep-kernel ablation timings (diagnostic builds from variants/, results
# wrong by construction): fluA bench kernel time per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abl}; mkdir -p $O
for v in "$@"; do
  [ "$v" = "$1" ] && continue
  PHYLO_HIP_LIB=variants/libphylo_hip_$v.so timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/fluA_$v.json 2> $O/fluA_$v.log || exit 1
  python -c "import json,sys; r=json.loads(open('$O/fluA_$v.json').read().strip().splitlines()[-1]); print('$v', r['roofline']['kernel_avg_ms'], r['value'])"
done
echo ALLDONE
