# fluA sweep time + PMC traffic per library variant from variants/ (run through gpurun): $1 = tag, then variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-varpmc}; mkdir -p $O; shift
for v in "$@"; do
  PHYLO_HIP_LIB=variants/libphylo_hip_$v.so timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/fluA_$v.json 2> $O/fluA_$v.log || exit 1
  PHYLO_HIP_LIB=variants/libphylo_hip_$v.so timeout -k 10 300 python tools/pmc_traffic.py --workload fluA --out $O/pmc_$v.json --scratch $O/pmc_$v > $O/pmc_$v.log 2>&1 || exit 1
  python -c "import json; r=json.loads(open('$O/fluA_$v.json').read().strip().splitlines()[-1]); p=json.load(open('$O/pmc_$v.json')); print('$v', round(r['roofline']['kernel_avg_ms'],4), round(r['value']), list(p['per_launch_bytes'].values())[0]/1e9)"
done
echo ALLDONE
