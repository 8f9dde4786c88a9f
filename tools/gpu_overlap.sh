# Two-context overlap probe and config 5 with one / two chain groups.
#   gpurun --timeout 600 -- bash tools/gpu_overlap.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ovl}; mkdir -p $O
timeout -k 10 120 python tools/overlap_probe.py resident 2 > $O/ovl.jsonl 2> $O/ovl.err && \
timeout -k 10 120 python tools/overlap_probe.py pattern 2 >> $O/ovl.jsonl 2>> $O/ovl.err && \
timeout -k 10 150 python tools/run_config5.py --groups 1 --out $O/g1 > $O/g1.log 2>&1 && \
timeout -k 10 150 python tools/run_config5.py --groups 2 --out $O/g2 > $O/g2.log 2>&1 && echo ALLDONE
cat $O/ovl.jsonl
for g in g1 g2; do python -c "import json; r=json.load(open('$O/$g/config5.json')); print('$g', r['engine'], r['chain_groups'], round(r['wall_s'],2))"; done
