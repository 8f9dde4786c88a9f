# Small-batch latency per engine (draws per call 1 / 4 / 16).
#   gpurun --timeout 600 -- bash tools/gpu_latency_engines.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-late}; mkdir -p $O
for w in fluA HCV; do for e in pattern resident; do for n in 1 4 16; do
  timeout -k 10 120 python tools/latency_probe.py --workload $w --engine $e --draws $n --calls 200 >> $O/lat.jsonl 2>> $O/lat.err || exit $?
done; done; done
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/rp -o run --output-format csv -- python tools/latency_probe.py --engine resident --draws 4 --calls 100 > $O/rp.log 2>&1 && echo ALLDONE
cat $O/lat.jsonl
