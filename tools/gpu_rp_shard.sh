# rocprofv3 kernel trace of the synthetic shard projection (run through gpurun); $1 = tag, $2 = shards
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rpshard}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp -o run --output-format csv -- python bench.py --workload synthetic --shard-of ${2:-8} --steps 10 --warmup 2 --no-cpu-baseline > $O/rp.log 2>&1 && echo ALLDONE
