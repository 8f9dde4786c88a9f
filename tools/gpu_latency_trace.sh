# Small-batch latency (the NUTS round shape) and its kernel trace.
#   gpurun --timeout 600 -- bash tools/gpu_latency_trace.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-lat}; mkdir -p $O
timeout -k 10 200 python tools/latency_probe.py --draws 4 > $O/probe.json 2> $O/probe.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/rp -o run --output-format csv -- python tools/latency_probe.py --draws 4 --calls 100 > $O/rp.log 2>&1 && echo ALLDONE
cat $O/probe.json
