# rocprofv3 kernel trace of the synthetic bench (run through gpurun); $1 = tag
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rpsyn}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp -o run --output-format csv -- python bench.py --workload synthetic --steps 10 --warmup 2 --no-cpu-baseline > $O/syn_rp.log 2>&1 && echo ALLDONE
