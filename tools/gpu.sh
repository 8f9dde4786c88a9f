#!/bin/bash
# GPU session script (run through gpurun from the repository root).
#   tools/gpu.sh TAG [step ...]      (steps below, run in the order given; default: tests bench shard8 synth multidev)
# A/B steps read their variants from AB_VARIANTS, a space-separated list whose
# items are `base` (this build), a variant library `variants/x.so` (loaded with
# PHYLO_HIP_AB=1 PHYLO_HIP_LIB), or environment settings `K=V[,K=V...]` for
# this build; they alternate the variants, two rounds (AB_REPS):
#   AB_VARIANTS="base variants/x.so PHY_PAIR=0" AB_ARGS="--workload synthetic --shard-of 8" tools/gpu.sh T ab
#   AB_VARIANTS="base variants/x.so" LAT_WLS="fluA HCV" LAT_DRAWS="4 100" tools/gpu.sh T latab
#   tools/gpu.sh T infer | draws | ldsenv     (the round-2/3 inference, draws-per-launch and LDS-plan runs)
# Every GPU step has its own time limit and the steps are chained: the first
# failure ends the script (set -e), nothing is retried.  Outputs under
# gpurun_out/TAG/.
set -eo pipefail
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp

step_tests() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -40 $O/pytest.log
}
step_smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -3 $O/smoke.log
}
step_bench() {
  timeout -k 10 400 python bench.py --json-out $O/bench_fluA.json > $O/bench_fluA.log 2>&1
  tail -c 1500 $O/bench_fluA.json
}
step_rehearse() {  # the N = 2 path of the default run on the one GPU (gloo, both ranks on device 0)
  timeout -k 10 500 python bench.py --gpus 2 --rehearse --steps 20 --warmup 5 --json-out $O/bench_rehearse2.json \
    > $O/bench_rehearse2.log 2>&1 || { tail -30 $O/bench_rehearse2.log; exit 1; }
  tail -c 2500 $O/bench_rehearse2.json
}
step_parity() {  # the parity suites of the pattern sweep (every plan) and the configs
  timeout -k 10 600 python -u -m pytest tests/test_gpu_00_configs.py tests/test_gpu_parity.py tests/test_gpu_large_cb.py \
    -x -q --timeout 240 --timeout-method thread -k "not synthetic_full_size and not config5" \
    > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
  tail -15 $O/pytest_parity.log
}
vname() {  # file-name tag of a variant spec
  case $1 in base) echo base ;; *.so) basename $1 .so ;; *.so:*) echo "$(basename ${1%%:*} .so)_$(echo ${1#*:} | tr ',=/' '__-')" ;;
    *) echo "$1" | tr ',=/' '__-' ;; esac
}
vrun() {  # vrun SPEC cmd... : the command under that variant (SPEC: base, x.so, x.so:K=V[,K=V], K=V[,K=V])
  local v=$1; shift
  case $v in
    base) "$@" ;;
    *.so) PHYLO_HIP_AB=1 PHYLO_HIP_LIB=$PWD/$v "$@" ;;
    *.so:*) env $(echo "${v#*:}" | tr ',' ' ') PHYLO_HIP_AB=1 PHYLO_HIP_LIB=$PWD/${v%%:*} "$@" ;;
    *) env $(echo "$v" | tr ',' ' ') "$@" ;;
  esac
}
step_ab() {  # bench.py A/B: AB_ARGS over AB_VARIANTS (see the header), alternating
  for r in $(seq 1 ${AB_REPS:-2}); do
    for v in ${AB_VARIANTS:-base}; do
      n=$(vname $v)
      vrun $v timeout -k 10 300 python bench.py ${AB_ARGS:-} --no-cpu-baseline --json-out $O/ab_${n}_$r.json \
        > $O/ab_${n}_$r.log 2>&1 || { tail -20 $O/ab_${n}_$r.log; exit 1; }
      python -c "import json;d=json.load(open('$O/ab_${n}_$r.json'));r=d.get('roofline',{});print('$n rep$r', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'))"
    done
  done
}
step_latab() {  # sampler-call latency A/B: LAT_WLS x LAT_DRAWS over AB_VARIANTS, alternating, then a kernel trace per variant
  local V=${AB_VARIANTS:-base variants/r03.so variants/r04.so}
  for d in ${LAT_DRAWS:-100 4 1}; do
    for r in $(seq 1 ${AB_REPS:-2}); do
      for w in ${LAT_WLS:-fluA}; do
        for v in $V; do
          n=$(vname $v)
          vrun $v timeout -k 10 120 python tools/latency_probe.py --workload $w --draws $d --engine pattern \
            > $O/lat_${n}_${w}_${d}_$r.log 2>&1 || { tail -20 $O/lat_${n}_${w}_${d}_$r.log; exit 1; }
          echo "$n $w draws=$d rep$r $(tail -1 $O/lat_${n}_${w}_${d}_$r.log)"
        done
      done
    done
  done
  [ -n "${LAT_TRACE-1}" ] || return 0
  local d=${LAT_TRACE_DRAWS:-100}
  for v in $V; do  # that call's kernels on the device clock
    n=$(vname $v)
    vrun $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_lat${d}_$n -o run -- \
      python tools/latency_probe.py --workload fluA --draws $d --engine pattern > $O/prof_lat${d}_$n.log 2>&1
    echo "== $n"; python tools/prof_stats.py $O/prof_lat${d}_$n/run_results.db | head -8
  done
}
step_infer() {  # the inference tests and config 5 (full NUTS on fluA, GPU gradients)
  timeout -k 10 600 python -u -m pytest tests/test_gpu_class.py tests/test_gpu_inference.py -x -v --timeout 400 \
    --timeout-method thread > $O/pytest_inf.log 2>&1 || { tail -30 $O/pytest_inf.log; exit 1; }
  tail -12 $O/pytest_inf.log
  timeout -k 10 300 python tools/run_config5.py --out $O/config5 > $O/config5.log 2>&1
  tail -1 $O/config5.log
}
step_draws() {  # fluA throughput against draws per launch, alternating
  for r in 1 2; do for n in 8192 16384 32768; do
    timeout -k 10 200 python bench.py --draws $n --steps $((1638400 / n)) --warmup 5 --no-cpu-baseline --no-synthetic \
      --json-out $O/d${n}_$r.json > $O/d${n}_$r.log 2>&1
    python -c "import json;d=json.load(open('$O/d${n}_$r.json'));print('draws $n rep$r', round(d['value']), round(d['roofline']['kernel_avg_ms'],3))"
  done; done
}
step_ldsenv() {  # LDS plans through the environment (one-chunk budget, deep-stack variants)
  for e in - PHY_LDS_BUDGET=163840 PHY_LDS_BUDGET=163840,PHY_DEEP=2 PHY_DEEP=2; do
    [ $e = - ] && v=base || v=$e
    n=$(vname $v)
    vrun $v timeout -k 10 200 python bench.py --no-cpu-baseline --no-synthetic --steps 100 --warmup 10 \
      --json-out $O/lds_$n.json > $O/lds_$n.log 2>&1
    python -c "import json;d=json.load(open('$O/lds_$n.json'));p=d['program'];print('$n', round(d['value']), round(d['roofline']['kernel_avg_ms'],3), p['n_chunks'], p['matrices_per_chunk'], p['lds_bytes'], p['deep_lds_entries'], p['recomputed'])"
  done
}
step_shard8() {
  timeout -k 10 300 python bench.py --workload synthetic --shard-of 8 --steps 100 --warmup 10 \
    --no-cpu-baseline --json-out $O/bench_shard8.json > $O/bench_shard8.log 2>&1
  python -c "import json;d=json.load(open('$O/bench_shard8.json'));print('shard8', d['value'], d['ms_per_step'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_shard8 -o run -- \
    python bench.py --workload synthetic --shard-of 8 --steps 50 --warmup 5 --no-cpu-baseline \
    > $O/prof_shard8.log 2>&1
  python tools/eval_timeline.py $O/prof_shard8/run_results.db > $O/timeline_shard8.txt && tail -22 $O/timeline_shard8.txt
}
step_synth() {
  timeout -k 10 300 python bench.py --workload synthetic --steps 50 --warmup 5 --no-cpu-baseline \
    --json-out $O/bench_synth.json > $O/bench_synth.log 2>&1
  python -c "import json;d=json.load(open('$O/bench_synth.json'));print('synth', d['value'], d['ms_per_step'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_synth -o run -- \
    python bench.py --workload synthetic --steps 30 --warmup 5 --no-cpu-baseline > $O/prof_synth.log 2>&1
  python tools/eval_timeline.py $O/prof_synth/run_results.db > $O/timeline_synth.txt && tail -22 $O/timeline_synth.txt
}
step_multidev() {
  timeout -k 10 300 python bench.py --workload synthetic --multi-device 1 --steps 30 --warmup 5 \
    --no-cpu-baseline --json-out $O/bench_multidev1.json > $O/bench_multidev1.log 2>&1
  python -c "import json;d=json.load(open('$O/bench_multidev1.json'));print('multidev1', d['value'], d['config']['parallelism'])"
}
step_prof() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fluA -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sampler-latency --no-synthetic > $O/prof_fluA.log 2>&1
  python tools/prof_stats.py $O/prof_fluA/run_results.db | head -6
}
step_lat() {  # small calls: quad sweep against the column sweeps (PHY_QUAD=0)
  for w in fluA HCV DS1; do
    for d in 1 4 16 32; do
      for q in 1 0; do
        PHY_QUAD=$q timeout -k 10 120 python tools/latency_probe.py --workload $w --draws $d --engine pattern \
          > $O/lat_${w}_${d}_q$q.log 2>&1 && tail -1 $O/lat_${w}_${d}_q$q.log | sed "s/^/$w d=$d quad=$q /"
      done
    done
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_lat4 -o run -- \
    python tools/latency_probe.py --workload fluA --draws 4 --engine pattern > $O/prof_lat4.log 2>&1
}
step_lat4() {  # the sampler's call only (4 draws), every engine, plus its kernel trace
  for w in fluA HCV DS1; do
    for q in 1 0; do
      PHY_QUAD=$q timeout -k 10 120 python tools/latency_probe.py --workload $w --draws 4 --engine pattern \
        > $O/lat4_${w}_q$q.log 2>&1 && tail -1 $O/lat4_${w}_q$q.log | sed "s/^/$w d=4 quad=$q /"
    done
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_lat4 -o run -- \
    python tools/latency_probe.py --workload fluA --draws 4 --engine pattern > $O/prof_lat4.log 2>&1
  python tools/prof_stats.py $O/prof_lat4/run_results.db
}
step_sq4() {  # SQ counters of the (multi-wave) quad sweep on the 4-draw fluA call (separate --pmc passes)
  PMC_SCRIPT=tools/latency_probe.py PMC_KERNEL=qmw timeout -k 10 600 python tools/pmc_sq.py \
    --workload fluA --draws 4 --engine pattern --calls 50 > $O/sq4_qsweep.json 2> $O/sq4_qsweep.err
  PMC_SCRIPT=tools/latency_probe.py PMC_KERNEL=qfin timeout -k 10 600 python tools/pmc_sq.py \
    --workload fluA --draws 4 --engine pattern --calls 50 > $O/sq4_qfin.json 2> $O/sq4_qfin.err
  head -c 600 $O/sq4_qsweep.json
}
step_shardn() {  # the shard-of-8 evaluation with batched draws (4 NUTS chains / 8 / 16 per call)
  for d in 4 8 16; do
    timeout -k 10 300 python bench.py --workload synthetic --shard-of 8 --draws $d --steps 50 --warmup 5 \
      --no-cpu-baseline --json-out $O/bench_shard8_d$d.json > $O/bench_shard8_d$d.log 2>&1
    python -c "import json;d=json.load(open('$O/bench_shard8_d$d.json'));print('shard8 draws=$d', d['value'], d['ms_per_step'])"
  done
  timeout -k 10 300 python bench.py --workload synthetic --draws 4 --steps 20 --warmup 3 --no-cpu-baseline \
    --json-out $O/bench_synth_d4.json > $O/bench_synth_d4.log 2>&1
  python -c "import json;d=json.load(open('$O/bench_synth_d4.json'));print('synth draws=4', d['value'], d['ms_per_step'])"
}
step_lines() {  # the committed bench lines: every dataset with its CPU baseline
  for w in HCV DS1 synthetic; do
    timeout -k 10 500 python bench.py --workload $w --json-out $O/bench_$w.json > $O/bench_$w.log 2>&1
    python -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w', d['value'], d['ms_per_step'], d['cpu_baseline']['value'])"
  done
}
step_profn() {  # kernel traces of the batched-draw class sweep (4 draws per call)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_shard8_d4 -o run -- \
    python bench.py --workload synthetic --shard-of 8 --draws 4 --steps 30 --warmup 5 --no-cpu-baseline \
    > $O/prof_shard8_d4.log 2>&1
  python tools/prof_stats.py $O/prof_shard8_d4/run_results.db | head -16
}
step_pmc() {  # HBM traffic (FETCH / WRITE passes) and SQ counters of the timed kernels, fluA and synthetic
  timeout -k 10 600 python tools/pmc_traffic.py --workload fluA > $O/pmc_traffic_fluA.log 2>&1 && tail -1 $O/pmc_traffic_fluA.log
  timeout -k 10 600 python tools/pmc_sq.py --steps 3 --warmup 1 --no-cpu-baseline --no-sampler-latency --no-synthetic \
    > $O/sq_pattern_fluA.json 2> $O/sq_pattern_fluA.err && head -c 400 $O/sq_pattern_fluA.json
  timeout -k 10 600 python tools/pmc_traffic.py --workload synthetic --engine class > $O/pmc_traffic_synth.log 2>&1 \
    && tail -1 $O/pmc_traffic_synth.log
  timeout -k 10 600 python tools/pmc_sq.py --workload synthetic --engine class --steps 3 --warmup 1 --no-cpu-baseline \
    --no-sampler-latency > $O/sq_class_synthetic.json 2> $O/sq_class_synthetic.err && head -c 400 $O/sq_class_synthetic.json
  cp profiles/pmc_traffic.json profiles/sq_counters.json $O/
}

STEPS=("$@")
[ ${#STEPS[@]} -eq 0 ] && STEPS=(tests bench shard8 synth multidev)
for st in "${STEPS[@]}"; do
  declare -F "step_$st" > /dev/null || { echo "unknown step $st"; exit 2; }
  echo "== step $st ($(date +%T))"
  "step_$st"
done
echo done
