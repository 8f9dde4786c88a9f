#!/usr/bin/env python
"""Full-rank ADVI on fluA (the GPU test's model, -q fullrank, the reference's
defaults) on the CPU with the C port as the likelihood (tests/cport_rows.py):
which runs converge near the README posterior and which stop early, and
what decides it.  TEST INFRASTRUCTURE (calls oracle/).  tests/test_fullrank_fate.py
holds the short, asserted versions; DESIGN.md 11 the measured table.

    python -m tools.fullrank_sensitivity --seeds 1,2,3 [--eta 0.1] [--threads 1]
    python -m tools.fullrank_sensitivity --trials 8 [--eps 2.2e-16]      # perturbed gradients, seed --seed
    python -m tools.fullrank_sensitivity --adapt-only --trials 12        # the adaptation's draw counts

Trial 0 is unperturbed; trial k > 0 multiplies every gradient entry of every
likelihood row by (1 + eps u), u uniform in {-1, 0, 1} (seeded by k).  Prints
one JSON line per run: eta, iterations, final ELBO, the clock rate's and
kappa's posterior means, converged or capped (or, with --adapt-only, eta,
the gradient / ELBO draws the adaptation consumed and a hash of the generator
state SGA starts from).
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--eps", type=float, default=2.0 ** -52)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--iter", type=int, default=100000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="/tmp/fullrank_sens")
    ap.add_argument("--eta", type=float, help="fixed eta (no adaptation, as run --eta)")
    ap.add_argument("--adapt-only", action="store_true",
                    help="stop at the start of SGA; print the adaptation's draw counts and the RNG state")
    ap.add_argument("--seeds", help="comma list of -S seeds, one unperturbed run each (instead of --trials)")
    a = ap.parse_args()
    from phylostan_amd import stan_io
    from tests.cport_rows import fluA_fullrank
    plan = ([(0, int(x)) for x in a.seeds.split(",")] if a.seeds else
            [(trial, a.seed) for trial in range(a.first, a.first + a.trials)])
    for trial, seed in plan:
        eps = 0.0 if trial == 0 else a.eps
        out = os.path.join(a.out, "s%d_t%d" % (seed, trial))
        t0 = time.time()
        lines, trace, state = fluA_fullrank(out, seed, a.iter, eta=a.eta, eps=eps, pert_seed=trial,
                                            nthreads=a.threads, stop_sga=a.adapt_only)
        rec = {"trial": trial, "seed": seed, "eps": eps, "seconds": time.time() - t0}
        if a.adapt_only:
            rec.update(eta=state["eta"], n_grad=state["n_grad"], n_lp=state["n_lp"],
                       rng=hashlib.sha1(state["rng"].encode()).hexdigest()[:12])
        else:
            prog = [ln for ln in lines if ln.strip()[:1].isdigit()]
            header, data = stan_io.read_samples(os.path.join(out, "fr"))
            col = {n: k for k, n in enumerate(header)}
            eta = [ln for ln in lines if ln.startswith("Success!")]
            rec.update(eta=eta[-1] if eta else a.eta, iterations=int(prog[-1].split()[0]), final_elbo=trace[-1],
                       converged="CONVERGED" in prog[-1], rate_mean=float(data[1:, col["rate"]].mean()),
                       kappa_mean=float(data[1:, col["kappa"]].mean()), elbo_trace=trace)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
