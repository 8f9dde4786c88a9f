set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01e; mkdir -p $O
timeout -k 10 300 python -m pytest tests/ -q -m gpu > $O/pytest.log 2>&1; tail -3 $O/pytest.log
B="timeout -k 10 200 python bench.py --no-cpu-baseline"
S="timeout -k 10 200 python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline"
V=$PWD/phylostan_amd/variants
$B > $O/fluA_out.json 2>&1; $B --cols 1 > $O/fluA_out_k1.json 2>&1
PHYLO_HIP_LIB=$V/inline.so $B > $O/fluA_in.json 2>&1; PHYLO_HIP_LIB=$V/inline.so $B --cols 1 > $O/fluA_in_k1.json 2>&1
$S > $O/syn_out.json 2>&1; PHYLO_HIP_LIB=$V/inline.so $S > $O/syn_in.json 2>&1
for f in $O/*.json; do python -c "
import json,sys
try:
    d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline']['kernel_avg_ms'],3), round(d['roofline']['frac'],3), d['program']['cols'])
except Exception as e: print('$f', 'ERR', open('$f').read()[-300:])
"; done
