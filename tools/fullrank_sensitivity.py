#!/usr/bin/env python
"""Full-rank ADVI on fluA (the GPU test's run: -q fullrank, seed 1, the
reference's defaults) on the CPU, with the C port as the likelihood and the
gradient rows perturbed at the last-bit level: does the trajectory's fate
(converged near the README point, or stalled in another mode) depend on
rounding?  TEST INFRASTRUCTURE (calls oracle/).

    python -m tools.fullrank_sensitivity [--trials 8] [--eps 2.2e-16] [--threads 8]

Trial 0 is unperturbed; trial k > 0 multiplies every gradient entry of every
likelihood row by (1 + eps u), u uniform in {-1, 0, 1} (seeded by k).  Prints
one JSON line per trial: eta, iterations, final ELBO, the clock rate's and
kappa's posterior means, converged or capped.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


class CPortRows:
    """evaluate_rows through the C port (compact rows), optionally perturbed."""

    def __init__(self, tipcodes, weights, peel0, rooted, model, C, eps=0.0, seed=0, nthreads=8, **_):
        from oracle import numpy_pruner as npr
        self.tip, self.w, self.peel0, self.rooted, self.C = tipcodes, weights, peel0, rooted, C
        self.kind = npr.MODEL_IDS[model]
        self.S = tipcodes.shape[0]
        self.B = 2 * self.S - 2 if rooted else 2 * self.S - 3
        self.eps, self.rng, self.nt = eps, np.random.default_rng(seed), nthreads

    def evaluate_rows(self, blens, mv):
        from oracle import cpu
        o = 1 + self.B + 2 * self.C + 14
        rows = np.stack([cpu.evaluate(self.tip, self.w, self.peel0, self.rooted, self.kind, mv[k], blens[k], self.C,
                                      nthreads=self.nt)[0][:o] for k in range(blens.shape[0])])
        if self.eps:
            u = self.rng.integers(-1, 2, rows[:, 1:].shape)
            rows[:, 1:] *= 1.0 + self.eps * u
        return rows

    def close(self):
        pass


def _adapt_only(a):
    """Eta adaptation only (trial k > 0 perturbed as above): the number of
    gradient / ELBO draws it consumed, the dropped ones, and a hash of the
    generator state SGA starts from -- SGA restarts from q0 (advi.py run), so
    that state and eta are all it inherits from the adaptation."""
    import hashlib
    from phylostan_amd import advi, cli
    from tests import fixture_files
    t, aln = fixture_files.write_dataset("fluA", a.out)
    import argparse as _ap

    class Stop(Exception):
        pass

    state = {}
    orig_grad = advi.ADVI.calc_elbo_grad

    def counting_grad(self, q):
        before = self.n_grad
        r = orig_grad(self, q)
        state["drops"] = state.get("drops", 0) + (self.n_grad - before - self.grad_samples)
        return r

    def stop_sga(self, q, eta, *x, **k):
        bg = self.rng.bit_generator.state
        state.update(eta=eta, n_grad=self.n_grad, n_lp=self.n_lp,
                     rng=hashlib.sha1(repr(bg).encode()).hexdigest()[:12])
        raise Stop()

    advi.ADVI.calc_elbo_grad = counting_grad
    advi.ADVI.sga = stop_sga
    for trial in range(a.first, a.first + a.trials):
        eps = 0.0 if trial == 0 else a.eps
        state.clear()
        parser = _ap.ArgumentParser()
        sub = parser.add_subparsers()
        cli.create_run_parser(sub).set_defaults(func=cli.run)
        arg = parser.parse_args(["run", "-s", os.path.join(a.out, "fluA.json"), "-m", "HKY", "-C", "4",
                                 "--heterochronous", "--estimate_rate", "--clock", "strict", "--coalescent",
                                 "constant", "-i", aln, "-t", t, "-o", os.path.join(a.out, "ad%d" % trial),
                                 "-q", "fullrank", "-S", str(a.seed)])
        try:
            cli.run(arg, likelihood_factory=lambda *x, **k: CPortRows(*x, eps=eps, seed=trial, nthreads=a.threads),
                    log=lambda *_: None)
        except Stop:
            pass
        print(json.dumps(dict(trial=trial, eps=eps, **state)), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--eps", type=float, default=2.0 ** -52)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--iter", type=int, default=100000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="/tmp/fullrank_sens")
    ap.add_argument("--eta", type=float, help="fixed eta (no adaptation, as run --eta)")
    ap.add_argument("--adapt-only", action="store_true",
                    help="stop at the start of SGA; print the adaptation's draw counts and the RNG state")
    ap.add_argument("--seeds", help="comma list of -S seeds, one unperturbed trial each (instead of --trials)")
    a = ap.parse_args()
    import argparse as _ap
    from phylostan_amd import cli, stan_io
    from tests import fixture_files
    os.makedirs(a.out, exist_ok=True)
    if a.adapt_only:
        _adapt_only(a)
        return
    t, aln = fixture_files.write_dataset("fluA", a.out)
    plan = ([(0, int(x)) for x in a.seeds.split(",")] if a.seeds else
            [(trial, a.seed) for trial in range(a.first, a.first + a.trials)])
    for trial, seed in plan:
        eps = 0.0 if trial == 0 else a.eps
        parser = _ap.ArgumentParser()
        sub = parser.add_subparsers()
        cli.create_run_parser(sub).set_defaults(func=cli.run)
        out = os.path.join(a.out, "fr%d" % trial)
        arg = parser.parse_args(["run", "-s", os.path.join(a.out, "fluA.json"), "-m", "HKY", "-C", "4",
                                 "--heterochronous", "--estimate_rate", "--clock", "strict", "--coalescent",
                                 "constant", "-i", aln, "-t", t, "-o", out, "-q", "fullrank", "-S", str(seed),
                                 "--iter", str(a.iter)] + (["--eta", str(a.eta)] if a.eta else []))
        lines = []
        t0 = time.time()
        cli.run(arg, likelihood_factory=lambda *x, **k: CPortRows(*x, eps=eps, seed=trial, nthreads=a.threads),
                log=lines.append)
        el = time.time() - t0
        prog = [ln for ln in lines if ln.strip()[:1].isdigit()]
        last = prog[-1].split()
        header, data = stan_io.read_samples(out)
        col = {n: k for k, n in enumerate(header)}
        eta = [ln for ln in lines if ln.startswith("Success!")]
        rec = {"trial": trial, "seed": seed, "eps": eps, "eta": eta[-1] if eta else None, "iterations": int(last[0]),
               "final_elbo": float(last[1]), "converged": "CONVERGED" in prog[-1],
               "rate_mean": float(data[1:, col["rate"]].mean()), "kappa_mean": float(data[1:, col["kappa"]].mean()),
               "seconds": el, "elbo_trace": [float(ln.split()[1]) for ln in prog]}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
