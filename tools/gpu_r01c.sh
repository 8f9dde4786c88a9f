set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01c; mkdir -p $O
timeout -k 10 300 python -m pytest tests/ -q -m gpu -x > $O/pytest.log 2>&1; tail -15 $O/pytest.log
B="timeout -k 10 200 python bench.py --no-cpu-baseline"
S="timeout -k 10 200 python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline"
$B > $O/fluA_auto.json 2>&1; $B --cols 1 > $O/fluA_k1.json 2>&1; $B --cols 2 --lds-budget 163840 > $O/fluA_k2_160.json 2>&1
PHYLO_HIP_LIB=$PWD/phylostan_amd/variants/wpe2.so $B --cols 2 > $O/fluA_k2_wpe2.json 2>&1
$S > $O/syn_auto.json 2>&1; $S --cols 2 --lds-budget 163840 > $O/syn_k2_160.json 2>&1; $S --cols 1 --lds-budget 163840 > $O/syn_k1_160.json 2>&1
PHYLO_HIP_LIB=$PWD/phylostan_amd/variants/wpe2.so $S --cols 2 --lds-budget 163840 > $O/syn_k2_160_wpe2.json 2>&1
for f in $O/*.json; do python -c "
import json,sys
try:
    d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value'],1), d['roofline']['kernel_avg_ms'], round(d['roofline']['frac'],3), d['program'])
except Exception as e: print('$f', 'ERR', open('$f').read()[-300:])
"; done
