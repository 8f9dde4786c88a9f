# SQ / TCC counter passes of the sweep kernel (tools/pmc_sq.py) on both
# bench workloads.  Run through gpurun:  gpurun -- bash tools/gpu_sq.sh [TAG] [LIB]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sq}; mkdir -p $O
[ -n "$2" ] && export PHYLO_HIP_LIB=$PWD/$2
timeout -k 10 600 python tools/pmc_sq.py --workload synthetic --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_syn.json 2> $O/sq_syn.err && cat $O/sq_syn.json &&
timeout -k 10 600 python tools/pmc_sq.py --steps 20 --warmup 2 --no-cpu-baseline > $O/sq_fluA.json 2> $O/sq_fluA.err && cat $O/sq_fluA.json
