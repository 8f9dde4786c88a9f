# Synthetic shard projections (bench.py --shard-of N, N = 2, 4, 8).
#   gpurun --timeout 600 -- bash tools/gpu_shards.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-shards}; mkdir -p $O
for n in 2 4 8; do timeout -k 10 300 python bench.py --workload synthetic --shard-of $n --steps 50 --warmup 5 --no-cpu-baseline --json-out $O/syn_shard$n.json > $O/syn_shard$n.log 2>&1 || exit $?; done
echo ALLDONE
