#!/bin/bash
# Same-box A/B: round-2 kernel (variants/r02.so) vs this tree (H=1 / auto);
# small-batch latency per engine / column plan; host profile of config 5.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ab2_r03; mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))
print(sys.argv[2], "evals/s %.0f kernel %.3f ms frac %.3f" % (r["value"], r["roofline"]["kernel_avg_ms"], r["roofline"]["frac"]))
PY
}
for rep in 1 2; do
  PHYLO_HIP_LIB=variants/r02.so timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-sampler-latency --json-out $O/r02_$rep.json > $O/r02_$rep.log 2>&1 && summ $O/r02_$rep.json r02_$rep || exit 1
  PHY_H=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-sampler-latency --json-out $O/h1_$rep.json > $O/h1_$rep.log 2>&1 && summ $O/h1_$rep.json h1_$rep || exit 1
done
for e in "pattern" "resident"; do
  for d in 1 4 100; do
    timeout -k 10 60 python tools/latency_probe.py --draws $d --calls 200 --engine $e >> $O/lat.jsonl 2>> $O/lat.err || exit 1
    PHY_COLS=1 PHY_H=1 timeout -k 10 60 python tools/latency_probe.py --draws $d --calls 200 --engine $e > $O/tmp.json 2>> $O/lat.err && sed 's/}/, "cols1_h1": true}/' $O/tmp.json >> $O/lat.jsonl || exit 1
    PHY_H=1 timeout -k 10 60 python tools/latency_probe.py --draws $d --calls 200 --engine $e > $O/tmp.json 2>> $O/lat.err && sed 's/}/, "h1": true}/' $O/tmp.json >> $O/lat.jsonl || exit 1
  done
done
cat $O/lat.jsonl
timeout -k 10 300 python -m cProfile -s tottime tools/run_config5.py --warmup 150 --samples 50 --engine pattern --out $O/c5 > $O/c5prof.txt 2>&1; head -60 $O/c5prof.txt | tail -45
