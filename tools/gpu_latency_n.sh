# Per-call latency vs draws per call, pattern and resident engines (fluA, HCV).
#   gpurun --timeout 600 -- bash tools/gpu_latency_n.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-latn}; mkdir -p $O
for w in fluA HCV; do for n in 32 64 100 256; do for e in pattern resident; do
  timeout -k 10 120 python tools/latency_probe.py --workload $w --engine $e --draws $n --calls 100 >> $O/lat.jsonl 2>> $O/lat.err || exit $?
done; done; done
cat $O/lat.jsonl
