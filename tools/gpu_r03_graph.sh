#!/bin/bash
# HIP graphs: parity tests, then small-call latency and the synthetic
# shard-8 projection with graphs on / off:  gpurun -- bash tools/gpu_r03_graph.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/graph_${1:-a}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for g in 1 0; do
  for e in pattern resident; do
    PHY_GRAPH=$g timeout -k 10 120 python tools/latency_probe.py --draws 4 --calls 400 --engine $e > $O/lat_${e}_g$g.log 2>&1 || exit $?
    echo "graph=$g $(cat $O/lat_${e}_g$g.log)"
  done
  PHY_GRAPH=$g timeout -k 10 300 python bench.py --workload synthetic --shard-of 8 --steps 100 --warmup 10 --no-cpu-baseline --json-out $O/shard8_g$g.json > $O/shard8_g$g.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('$O/shard8_g$g.json')); print('graph=$g shard8', round(d['value'],1), 'evals/s', 'kernel_ms', round(d['roofline']['kernel_avg_ms'],4))"
  PHY_GRAPH=$g timeout -k 10 300 python bench.py --workload synthetic --steps 30 --warmup 5 --no-cpu-baseline --json-out $O/syn_g$g.json > $O/syn_g$g.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('$O/syn_g$g.json')); print('graph=$g synthetic', round(d['value'],1), 'evals/s', 'kernel_ms', round(d['roofline']['kernel_avg_ms'],4))"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/rp_shard8 -o run --output-format csv -- \
  python bench.py --workload synthetic --shard-of 8 --steps 30 --warmup 5 --no-cpu-baseline --no-sampler-latency > $O/rp_shard8.log 2>&1
