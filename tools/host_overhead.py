"""Host-side cost of a NUTS round on config 5's model (fluA HKY+W4 strict
clock, constant coalescent), measured on the CPU with the C port standing in
for the GPU: the time per gradient round minus the stand-in's own time is
what the sampler, transforms, priors and chain rule cost per round.

Test infrastructure (it calls oracle/): run from the repository root as
    python -m tools.host_overhead [--warmup 60 --samples 60 --profile]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


class CPortLikelihood:
    """evaluate_rows through the C port (compact rows), timed."""

    def __init__(self, d, peel0, C, nthreads=1):
        self.tip, self.w, self.peel0, self.C, self.nt = d["tipbits"], d["weights"], peel0, C, nthreads
        self.B = 2 * d["tipbits"].shape[0] - 2
        self.seconds = 0.0
        self.calls = 0

    def evaluate_rows(self, blens, mv):
        from oracle import cpu
        t0 = time.perf_counter()
        o = 1 + self.B + 2 * self.C + 14
        rows = np.stack([cpu.evaluate(self.tip, self.w, self.peel0, True, 1, mv[k], blens[k], self.C,
                                      nthreads=self.nt)[0][:o] for k in range(blens.shape[0])])
        self.seconds += time.perf_counter() - t0
        self.calls += 1
        return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--samples", type=int, default=60)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    from phylostan_amd.nuts import run_chains
    from phylostan_amd.posterior import ModelSpec, Posterior, TreeData
    from tests import cases
    d = cases.load_layout("fluA")
    S = d["tipbits"].shape[0]
    peel0 = d["peel"] - 1
    tree = TreeData(S, peel0, d["map"], d["lowers"], float(d["oldest"]))
    spec = ModelSpec(model="HKY", categories=4, clock="strict", estimate_rate=True, coalescent="constant",
                     heterochronous=True)
    lik = CPortLikelihood(d, peel0, 4)
    post = Posterior(spec, tree, lik, compact_rows=True)
    q0s = [post.initial_point(np.random.default_rng((1, c))) for c in range(a.chains)]
    prof = cProfile.Profile() if a.profile else None
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    chains = run_chains(post, q0s, [(1, c) for c in range(a.chains)], num_warmup=a.warmup, num_samples=a.samples)
    if prof:
        prof.disable()
    el = time.perf_counter() - t0
    host = el - lik.seconds
    print("rounds %d, gradient evaluations %d, wall %.2f s, stand-in %.2f s -> host %.1f us per round"
          % (lik.calls, sum(c.n_grad for c in chains), el, lik.seconds, 1e6 * host / lik.calls))
    if prof:
        pstats.Stats(prof).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
