set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01b; mkdir -p $O
timeout -k 10 300 python -m pytest tests/ -q -m gpu > $O/pytest.log 2>&1; tail -3 $O/pytest.log
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/pf2_fluA.json 2>&1 && tail -c 700 $O/pf2_fluA.json
PHYLO_HIP_LIB=$PWD/phylostan_amd/variants/pf1.so timeout -k 10 200 python bench.py --no-cpu-baseline > $O/pf1_fluA.json 2>&1 && tail -c 700 $O/pf1_fluA.json
timeout -k 10 200 python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > $O/pf2_syn.json 2>&1 && tail -c 800 $O/pf2_syn.json
PHYLO_HIP_LIB=$PWD/phylostan_amd/variants/pf1.so timeout -k 10 200 python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > $O/pf1_syn.json 2>&1 && tail -c 800 $O/pf1_syn.json
timeout -k 10 600 python tools/pmc_sq.py > $O/sq_fluA.json 2> $O/sq_fluA.err; cat $O/sq_fluA.json
