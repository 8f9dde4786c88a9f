# fluA bench under several tuning flags:  gpurun -- bash tools/gpu_sweep.sh TAG "flags1" "flags2" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
i=0
for F in "$@"; do
  i=$((i+1))
  timeout -k 10 240 python bench.py --steps 50 --warmup 5 --no-cpu-baseline $F > $O/r$i.json 2> $O/r$i.err || exit $?
  echo "[$F] $(python -c "import json;d=json.load(open('$O/r$i.json'));print(d['value'],d['roofline']['frac'],d['program'])")"
done
