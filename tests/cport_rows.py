"""The C port (oracle/cpu_pruner.c) behind the engine's ``evaluate_rows``
interface, so the inference drivers (cli.run, ADVI, NUTS) can run on the CPU
with the oracle as their likelihood -- TEST INFRASTRUCTURE (calls oracle/),
used by tests/test_fullrank_fate.py and tools/fullrank_sensitivity.py.

``eps`` > 0 multiplies every gradient entry of every row by (1 + eps u), u
uniform in {-1, 0, 1} from a generator seeded by ``seed``: last-bit noise of
the size a different summation order gives.  ``nthreads`` = 1 makes the C
port's pattern sums (and so every row) deterministic."""
import os

import numpy as np

from tests import fixture_files

FLUA_RUN = ["-m", "HKY", "-C", "4", "--heterochronous", "--estimate_rate", "--clock", "strict", "--coalescent",
            "constant"]


class CPortRows:
    def __init__(self, tipcodes, weights, peel0, rooted, model, C, eps=0.0, seed=0, nthreads=1, **_):
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


def fluA_fullrank(outdir, seed, iters, eta=None, eps=0.0, pert_seed=0, nthreads=1, stop_sga=False):
    """``phylostan run -q fullrank`` on fluA (the GPU test's model) with the
    C port as the likelihood.  Returns (log lines, ELBO trace of the SGA
    progress lines, adapt state) -- with ``stop_sga`` the run ends where
    stochastic gradient ascent would start and the adapt state holds eta, the
    gradient / ELBO draws the adaptation consumed and the generator state."""
    import argparse
    from phylostan_amd import advi, cli
    os.makedirs(outdir, exist_ok=True)
    t, aln = fixture_files.write_dataset("fluA", outdir)
    parser = argparse.ArgumentParser()
    sub = parser.add_subparsers()
    cli.create_run_parser(sub).set_defaults(func=cli.run)
    arg = parser.parse_args(["run", "-s", os.path.join(outdir, "fluA.json")] + FLUA_RUN +
                            ["-i", aln, "-t", t, "-o", os.path.join(outdir, "fr"), "-q", "fullrank", "-S", str(seed),
                             "--iter", str(iters)] + (["--eta", repr(eta)] if eta else []))
    lines, state = [], {}

    class _Stop(Exception):
        pass

    orig = advi.ADVI.sga

    def stop(self, q, eta_, *a, **k):
        state.update(eta=eta_, n_grad=self.n_grad, n_lp=self.n_lp, rng=repr(self.rng.bit_generator.state))
        raise _Stop()

    if stop_sga:
        advi.ADVI.sga = stop
    try:
        cli.run(arg, likelihood_factory=lambda *x, **k: CPortRows(*x, eps=eps, seed=pert_seed, nthreads=nthreads),
                log=lines.append)
    except _Stop:
        pass
    finally:
        advi.ADVI.sga = orig
    trace = [float(ln.split()[1]) for ln in lines if ln.strip()[:1].isdigit()]
    return lines, trace, state
