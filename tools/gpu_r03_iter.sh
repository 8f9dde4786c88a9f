#!/bin/bash
# One build -> measure iteration:  gpurun -- bash tools/gpu_r03_iter.sh TAG
#   the -m gpu suite, small-call latency (auto plan, K=2, resident; the auto
#   plan under rocprof), the default bench line, the synthetic shard-8
#   projection.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/iter_${1:-a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -32 $O/tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/rp_lat -o run --output-format csv -- \
  python tools/latency_probe.py --draws 4 --calls 300 > $O/lat_auto.log 2>&1 && \
timeout -k 10 120 python tools/latency_probe.py --draws 4 --calls 300 >> $O/lat.log 2>&1 && \
timeout -k 10 120 python tools/latency_probe.py --draws 4 --calls 300 --cols 2 >> $O/lat.log 2>&1 && \
timeout -k 10 120 python tools/latency_probe.py --draws 4 --calls 300 --engine resident >> $O/lat.log 2>&1 && \
timeout -k 10 120 python tools/latency_probe.py --draws 1 --calls 300 >> $O/lat.log 2>&1 && \
cat $O/lat.log && \
timeout -k 10 300 python bench.py --json-out $O/fluA.json > $O/fluA.log 2>&1 && \
timeout -k 10 300 python bench.py --workload synthetic --shard-of 8 --steps 50 --warmup 5 --no-cpu-baseline --json-out $O/syn_shard8.json > $O/syn_shard8.log 2>&1 && \
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for f in ("fluA", "syn_shard8"):
    d = json.load(open("%s/%s.json" % (o, f)))
    print(f, "value %.1f" % d["value"], "kernel_ms %.4f" % d["roofline"]["kernel_avg_ms"], "frac %.3f" % d["roofline"]["frac"],
          "sampler", d.get("sampler_latency"), "draws_100", {k: v for k, v in (d.get("draws_100") or {}).items() if k != "note"})
PY
