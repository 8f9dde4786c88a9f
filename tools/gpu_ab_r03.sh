#!/bin/bash
# A/B of the sweep layout (PHY_H) and the single-launch path (PHY_DIRECT):
# fluA throughput (8192 draws) and small-batch latency (4 / 100 draws).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ab_r03; mkdir -p $O
run() {  # name, env..., -- args
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --json-out $O/$name.json > $O/$name.log 2>&1 || { tail -5 $O/$name.log; return 1; }
  python - "$O/$name.json" "$name" <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))
print(sys.argv[2], "evals/s %.0f kernel %.3f ms frac %.3f" % (r["value"], r["roofline"]["kernel_avg_ms"], r["roofline"]["frac"]),
      "lat4", {k: round(v, 1) for k, v in r["sampler_latency"].items() if k.endswith("call") and v},
      "d100", {k: round(v) for k, v in r["draws_100"].items() if k.endswith("call") and v}, "plan", r["program"]["lds_bytes"], r["program"]["n_chunks"])
PY
}
run h_auto && run h1 PHY_H=1 && run h_auto_nodirect PHY_DIRECT=0 && run h1_noqfuse PHY_H=1 PHY_QFUSE=0 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/rp_lat -o run --output-format csv -- python tools/latency_probe.py --draws 4 --calls 200 > $O/lat_rp.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/rp_lat_h1 -o run --output-format csv -- env PHY_H=1 python tools/latency_probe.py --draws 4 --calls 200 > $O/lat_rp_h1.log 2>&1 ; \
head -12 $O/rp_lat/*/run_kernel_stats.csv 2>/dev/null || find $O/rp_lat -name "*stats*" | head; echo ---; find $O/rp_lat_h1 -name "*kernel_stats.csv" -exec head -12 {} \; ; cat $O/lat_rp.log | tail -2
