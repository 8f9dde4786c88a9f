# Kernel trace of the synthetic 8-way shard projection (what each rank of an 8-GPU run computes).
#   gpurun --timeout 600 -- bash tools/gpu_shard_trace.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-shtrace}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp -o run --output-format csv -- python bench.py --workload synthetic --shard-of 8 --steps 10 --warmup 2 --no-cpu-baseline > $O/rp.log 2>&1 && echo ALLDONE
