"""Debug helper (test infrastructure, calls oracle/): the synthetic workload
on the GPU vs the C port, per output array, with the location of the
largest dL/dP error.  Run on the GPU box from the repository root:
    python -m tools.dbg_synthetic [n_sites] [engine ...]
PHYLO_HIP_LIB selects a variant library."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    from oracle import cpu
    from phylostan_amd import synthetic
    from phylostan_amd.engine import EvalResult, TreeLikelihood
    n_sites = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    engines = sys.argv[2:] or ["class", "pattern"]
    pd, prm = synthetic.simulate(n_sites=n_sites)
    mv = np.concatenate([prm["freqs"], prm["rates"], prm["rs"], prm["ps"]])
    nt = max(1, min(16, os.cpu_count() or 1))
    out, sl = cpu.evaluate(pd.tipcodes, pd.weights, pd.peel0, True, 2, mv, prm["blens"], 4, site_ll=True,
                           nthreads=nt)
    B = 2 * pd.tipcodes.shape[0] - 2
    ref = EvalResult(out, B, 4, sl)
    for engine in engines:
        eng = TreeLikelihood(pd.tipcodes, pd.weights, pd.peel0, True, "GTR", 4, max_draws=1)
        eng.set_engine(engine)
        res = eng.evaluate(prm["blens"], mv, site_ll=True)
        print("[%s] P=%d loglik %.17g ref %.17g" % (engine, pd.tipcodes.shape[1], res.loglik, ref.loglik))
        for k in ("dLdP", "grad_blens", "grad_rs", "grad_ps", "grad_freq_root", "grad_rates", "grad_freqs"):
            a, b = np.asarray(getattr(res, k)), np.asarray(getattr(ref, k))
            d = np.abs(a - b)
            i = np.unravel_index(np.argmax(d), d.shape)
            print("  %-15s rel %.2e  at %s: gpu %.17g ref %.17g  (max |ref| %.3g)"
                  % (k, d.max() / max(np.abs(b).max(), 1e-300), i, a[i], b[i], np.abs(b).max()))
        eng.close()


if __name__ == "__main__":
    main()
