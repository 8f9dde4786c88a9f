#!/usr/bin/env python
"""BASELINE.json config 5: full NUTS on fluA (HKY+W4, strict clock, constant
coalescent, heterochronous), 1000 warmup + 1000 draws per chain, every
leapfrog gradient from the GPU engine; posterior means / 95% intervals
compared with the reference's README.md:104-108 intervals.

Run on the GPU box:  python tools/run_config5.py [--chains 4] [--out DIR]
Writes DIR/fluA_nuts_{c}.csv (Stan format), DIR/config5.json (summary).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

README_CI = {"wshape": (0.383, 0.616), "rate": (0.00432, 0.00577), "theta": (3.14, 5.05),
             "kappa": (4.37, 7.039), "root_height": (18.36, 19.74)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--samples", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--engine", default="latency", choices=["latency", "auto", "pattern"],
                    help="latency: TreeLikelihood.prefer_latency_engine() (what the CLI uses for NUTS)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "config5"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    from phylostan_amd import stan_io
    from phylostan_amd.engine import TreeLikelihood
    from phylostan_amd.nuts import run_chains
    from phylostan_amd.posterior import ModelSpec, Posterior, TreeData
    from tests import cases

    d = cases.load_layout("fluA")
    S = d["tipbits"].shape[0]
    peel0 = d["peel"] - 1
    tree = TreeData(S, peel0, d["map"], d["lowers"], float(d["oldest"]))
    spec = ModelSpec(model="HKY", categories=4, clock="strict", estimate_rate=True, coalescent="constant",
                     heterochronous=True)
    def make_post():
        lik = TreeLikelihood(d["tipbits"], d["weights"], peel0, True, "HKY", 4, max_draws=a.chains)
        if a.engine == "latency":
            lik.prefer_latency_engine()
        elif a.engine != "auto":
            lik.set_engine(a.engine)
        return Posterior(spec, tree, lik, compact_rows=True)
    post = make_post()
    lik = post.lik
    q0s = [post.initial_point(np.random.default_rng((a.seed, c))) for c in range(a.chains)]
    t0 = time.time()
    chains = run_chains(post, q0s, [(a.seed, c) for c in range(a.chains)], num_warmup=a.warmup,
                        num_samples=a.samples, progress=lambda s: print(s, flush=True))
    el = time.time() - t0
    names = post.column_names()
    allrows = []
    for c, ch in enumerate(chains):
        rows = post.flat_rows(np.stack([dr[0] for dr in ch.draws]))
        path = os.path.join(a.out, "fluA_nuts_%d.csv" % c)
        stan_io.write_nuts_csv(path, names, ch, rows, [("model", "fluA HKY+W4 strict constant"), ("chain", c)],
                               elapsed=(el / 2, el / 2))
        allrows.append(rows[[not dr[8] for dr in ch.draws]])
    X = np.concatenate(allrows)
    col = {n: k for k, n in enumerate(names)}
    root = "heights.%d" % (S - 1)
    summ = {}
    for key, nm in [("wshape", "wshape"), ("rate", "rate"), ("theta", "theta"), ("kappa", "kappa"),
                    ("root_height", root)]:
        v = X[:, col[nm]]
        lo, hi = np.quantile(v, (0.025, 0.975))
        rlo, rhi = README_CI[key]
        summ[key] = {"mean": float(v.mean()), "ci95": [float(lo), float(hi)], "reference_ci95": [rlo, rhi],
                     "mean_within_reference_ci": bool(rlo <= v.mean() <= rhi)}
    n_grad = sum(ch.n_grad for ch in chains)
    rec = {"config": "fluA HKY+W4 strict clock, constant coalescent, NUTS %d chains x (%d warmup + %d draws)"
                     % (a.chains, a.warmup, a.samples),
           "engine": lik.engine(),
           "wall_s": el, "gradient_evaluations": n_grad, "grads_per_s": n_grad / el,
           "divergent": int(sum(dr[6] for ch in chains for dr in ch.draws if not dr[8])),
           "mean_accept": float(np.mean([dr[2] for ch in chains for dr in ch.draws if not dr[8]])),
           "mean_treedepth": float(np.mean([dr[4] for ch in chains for dr in ch.draws if not dr[8]])),
           "stepsize": [ch.eps for ch in chains], "summary": summ}
    with open(os.path.join(a.out, "config5.json"), "w") as fp:
        json.dump(rec, fp, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
