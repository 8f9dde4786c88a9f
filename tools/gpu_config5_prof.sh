# Config 5 under cProfile (host-side time split of the NUTS run).
#   gpurun --timeout 600 -- bash tools/gpu_config5_prof.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c5prof; mkdir -p $O
timeout -k 10 300 python -m cProfile -o $O/c5.prof tools/run_config5.py --out $O > $O/c5.log 2>&1 && \
python -c "
import pstats; p=pstats.Stats('$O/c5.prof'); p.sort_stats('cumulative').print_stats(45)" > $O/c5_cum.txt && \
python -c "
import pstats; p=pstats.Stats('$O/c5.prof'); p.sort_stats('tottime').print_stats(40)" > $O/c5_tot.txt && echo DONE
