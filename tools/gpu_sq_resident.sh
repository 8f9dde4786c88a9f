set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sqres; mkdir -p $O
PMC_KERNEL=res_rev_kernel timeout -k 10 400 python tools/pmc_sq.py --engine resident --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_rev.json 2> $O/sq_rev.err && \
PMC_KERNEL=res_fwd_kernel timeout -k 10 400 python tools/pmc_sq.py --engine resident --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_fwd.json 2> $O/sq_fwd.err && echo DONE
