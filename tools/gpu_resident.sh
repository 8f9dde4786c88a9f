# Resident class sweep: GPU parity tests, then fluA / HCV bench lines against the pattern sweep.
#   gpurun --timeout 900 -- bash tools/gpu_resident.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-res}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -v --timeout 120 --timeout-method thread > $O/test.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 200 python bench.py --engine resident --no-cpu-baseline --steps 50 --warmup 5 --json-out $O/fluA_res.json > $O/fluA_res.log 2>&1 && \
timeout -k 10 200 python bench.py --engine pattern --no-cpu-baseline --steps 50 --warmup 5 --json-out $O/fluA_pat.json > $O/fluA_pat.log 2>&1 && \
timeout -k 10 200 python bench.py --workload HCV --engine resident --no-cpu-baseline --steps 50 --warmup 5 --json-out $O/HCV_res.json > $O/HCV_res.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/rp -o run --output-format csv -- python bench.py --engine resident --no-cpu-baseline --steps 20 --warmup 3 > $O/rp.log 2>&1 && \
echo ALLDONE
tail -3 $O/test.log
for f in $O/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"; done
if [ "$2" = "sq" ]; then PMC_KERNEL=res_rev_kernel timeout -k 10 400 python tools/pmc_sq.py --engine resident --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_rev.json 2> $O/sq_rev.err; fi
