# A/B of an environment knob on the fluA bench (run through gpurun): $1 = tag, $2 = VAR, then values
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; V=$2; mkdir -p $O; shift 2
for x in "$@"; do
  env $V=$x timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/fluA_$x.json 2> $O/fluA_$x.log || exit 1
  python -c "import json; r=json.loads(open('$O/fluA_$x.json').read().strip().splitlines()[-1]); print('$V=$x', round(r['ms_per_step'],4), round(r['roofline']['kernel_avg_ms'],4), round(r['value']))"
done
echo ALLDONE
