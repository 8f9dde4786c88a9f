"""GPU parity of every BASELINE config, first in the -m gpu run.

This file sorts first so that, under ``pytest -x``, every config is checked
and recorded before any exploratory GPU test can stop the run.  Each test
records one line (tests/report.py) that the terminal summary prints:

  KAT        the reference's only known-answer test (eigen/test_ll_3tax.py)
  config 1   DS1 JC69 unrooted       -- reference-pinned (scripts/phylo.py, merged root edge)
  config 2   fluA HKY+W4 strict      -- reference-pinned (scripts/phylo.py per category, mixture)
  config 3   HCV GTR+W4              -- reference-pinned (same)
  phylo.py   four C = 1 HKY / GTR points of the reference's own pruner
  config 4   synthetic 128 x 1M GTR+W4 (528,111 patterns), full size, vs the C port
             (+ the class sweep at 200k sites)
  config 5   full NUTS on fluA, posterior means inside the README intervals

Tolerances: per-site / total log L rel 1e-10 (north_star asks 1e-6); every
gradient rel 1e-9 of its array's largest entry; the device exchangeability /
frequency gradients rel 1e-8 against the host chain rule on the oracle's dL/dP.
"""
import os

import numpy as np
import pytest

from tests import cases, report

pytestmark = pytest.mark.gpu

RTOL_LL = 1e-10
RTOL_G = 1e-9


def _engine(case, max_draws=1, **kw):
    from phylostan_amd.engine import TreeLikelihood
    return TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C,
                          max_draws=max_draws, **kw)


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _site_rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-2)))


def errors(res, ref, model):
    """Max relative errors of a GPU result against an oracle / C-port result."""
    e = {"site_ll": _site_rel(res.site_ll, ref["site_ll"]),
         "loglik": abs(res.loglik - ref["loglik"]) / abs(ref["loglik"])}
    for k in ("dLdP", "grad_blens", "grad_rs", "grad_ps", "grad_freq_root"):
        e[k] = _rel(getattr(res, k), ref[k])
    return e


def check(e, extra_q=None):
    assert e["site_ll"] <= RTOL_LL and e["loglik"] <= RTOL_LL, e
    for k in ("dLdP", "grad_blens", "grad_rs", "grad_ps", "grad_freq_root"):
        assert e[k] <= RTOL_G, (k, e)
    if extra_q is not None:
        assert extra_q <= 1e-8, extra_q


def q_param_error(case, res, ref):
    if case.model == "JC69":
        assert not np.any(res.grad_rates) and not np.any(res.grad_freqs)
        return 0.0
    from phylostan_amd import models
    gr, gf = models.q_param_gradients(ref["dLdP"], case.blens, case.rs, case.freqs, case.rates,
                                      ref["grad_freq_root"])
    return max(_rel(res.grad_rates, gr), _rel(res.grad_freqs, gf))


def fmt(e):
    return "site_ll %.1e  loglik %.1e  dLdP %.1e  grad_blens %.1e" % (e["site_ll"], e["loglik"], e["dLdP"],
                                                                      e["grad_blens"])


def test_kat_3tax_reference_values():
    """eigen/test_ll_3tax.py's closed form at its two points."""
    kat = cases.load_kat()
    worst_ll = worst_g = 0.0
    for pt in kat["points"]:
        case = cases.kat_case(pt)
        res = _engine(case).evaluate(case.blens, case.model_vec(), site_ll=True)
        check(errors(res, case.oracle(), case.model))
        worst_ll = max(worst_ll, abs(res.loglik - pt["loglik"]) / abs(pt["loglik"]))
        g = res.grad_blens * 0.75  # d/dt of the unnormalised-Q formula
        worst_g = max(worst_g, _rel(g[[0, 1, 3, 2]], pt["grad_fd"]))
        assert abs(res.loglik - pt["loglik"]) < 1e-12
        np.testing.assert_allclose(g[[0, 1, 3, 2]], pt["grad_fd"], rtol=1e-6)
    report.record("KAT 3-taxon (eigen/test_ll_3tax.py): loglik rel %.1e vs reference closed form, "
                  "grad rel %.1e vs its finite differences" % (worst_ll, worst_g))


MIXTURE_IDS = {"DS1": "config 1 DS1 JC69 unrooted", "fluA": "config 2 fluA HKY+W4",
               "HCV": "config 3 HCV GTR+W4"}


@pytest.mark.parametrize("k", range(3), ids=["DS1_JC69_unrooted", "fluA_HKY_W4", "HCV_GTR_W4"])
def test_config_vs_reference_pruner(k):
    """The configs' own likelihood variants against the reference's
    scripts/phylo.py (tests/golden/phylo_mixture.json): per-site and total
    log L at rel 1e-10; the full gradient against the oracle (finite-
    difference-pinned, tests/test_oracle.py) at 1e-9 / 1e-8."""
    pts = cases.load_mixture_points()
    order = ["DS1", "fluA", "HCV"]
    pt = [p for p in pts if p["dataset"] == order[k]][0]
    case = cases.mixture_case(pt)
    # the pattern sweep under both plans: one column per lane (what a
    # sampler's small context plans) and two (the batched bench's plan)
    for engine, cols in (("pattern", 1), ("pattern", 2), ("class", 0)):
        eng = _engine(case)
        eng.set_engine(engine)
        if cols:
            eng.set_tuning(cols=cols)
            assert eng.lds_plan()["cols"] == cols
        res = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
        ref = case.oracle()
        e = errors(res, ref, case.model)
        eq = q_param_error(case, res, ref)
        check(e, eq)
        e_ref_site = _site_rel(res.site_ll, pt["site_ll"])
        e_ref_ll = abs(res.loglik - pt["loglik"]) / abs(pt["loglik"])
        assert e_ref_site <= RTOL_LL and e_ref_ll <= RTOL_LL, (e_ref_site, e_ref_ll)
        report.record("%s [%s]: vs scripts/phylo.py loglik %.1e site_ll %.1e | vs oracle %s  Q-params %.1e"
                      % (MIXTURE_IDS[pt["dataset"]], engine + (" K=%d" % cols if cols else ""), e_ref_ll,
                         e_ref_site, fmt(e), eq))


@pytest.mark.parametrize("k", range(3), ids=["fluA_HKY_W4", "HCV_GTR_W4", "DS1_JC69_unrooted"])
def test_config_gradients_vs_reference_fd(k):
    """a9 pinned to the reference itself: the GPU's gradients (branch lengths,
    kappa or the six GTR exchangeabilities, the frequencies through Q plus the
    root term, the Weibull shape through dlogL/drs) against central
    differences of the reference's own likelihood (scripts/phylo.py per
    category, the mixture of generate_script.py:1006-1010;
    tests/golden/phylo_grad.json) at rel 1e-6, on both engines."""
    from tests.test_oracle import REF_GRAD_RTOL, reference_grad_errors, reference_grad_points
    pt = reference_grad_points()[k]
    mp = [p for p in cases.load_mixture_points() if p["dataset"] == pt["dataset"]][0]
    case = cases.mixture_case(mp)
    for engine in ("pattern", "class"):
        eng = _engine(case)
        eng.set_engine(engine)
        res = eng.evaluate(case.blens, case.model_vec())
        errs = reference_grad_errors({"grad_blens": res.grad_blens, "grad_rs": res.grad_rs,
                                      "grad_rates": res.grad_rates, "grad_freqs": res.grad_freqs}, pt, case)
        assert all(v <= REF_GRAD_RTOL for v in errs.values()), (engine, errs)
        report.record("%s [%s]: gradients vs reference finite differences: %s"
                      % (MIXTURE_IDS[pt["dataset"]], engine, "  ".join("%s %.1e" % kv for kv in errs.items())))


@pytest.mark.parametrize("k", range(4))
def test_reference_phylo_py_points(k):
    """HKY / GTR (C = 1) through the eigen path against scripts/phylo.py."""
    pt = cases.load_phylo_points()[k]
    case = cases.phylo_case(pt)
    res = _engine(case).evaluate(case.blens, case.model_vec(), site_ll=True)
    ref = case.oracle()
    e = errors(res, ref, case.model)
    eq = q_param_error(case, res, ref)
    check(e, eq)
    es = _site_rel(res.site_ll, pt["site_ll"])
    el = abs(res.loglik - pt["loglik"]) / abs(pt["loglik"])
    assert es <= RTOL_LL and el <= RTOL_LL
    report.record("phylo.py %s %s C=1: vs reference loglik %.1e site_ll %.1e | vs oracle %s"
                  % (pt["dataset"], pt["model"], el, es, fmt(e)))


def test_production_batch_fluA_every_row_vs_c_port():
    """The bench's shape: 1,024 distinct draws in ONE launch; 28 rows against
    the C port (log L, every gradient, dL/dP)."""
    from oracle import cpu
    from phylostan_amd import models
    base = cases.fluA_case()
    n = 1024
    eng = _engine(base, max_draws=n)
    rng = np.random.default_rng(17)
    blens = base.blens[None, :] * rng.uniform(0.5, 1.5, (n, base.blens.size))
    mvs = []
    for _ in range(n):
        f = rng.dirichlet([30.0] * 4)
        rs, ps = models.weibull_site_rates(rng.uniform(0.2, 2.0), base.C)
        mvs.append(models.model_vector(f, models.hky_exchangeabilities(rng.uniform(2.0, 9.0)), rs, ps))
    mvs = np.array(mvs)
    rows = eng.evaluate_rows(blens, mvs)
    B, C = eng.B, base.C
    o = 1 + B + 2 * C
    worst = [0.0, 0.0, 0.0, 0.0]
    for k in range(0, n, 37):
        ref, _ = cpu.evaluate(base.tipcodes, base.weights, base.peel0, True, 1, mvs[k], blens[k], base.C)
        got = rows[k]
        errs = [abs(got[0] - ref[0]) / abs(ref[0]), _rel(got[1:o + 4], ref[1:o + 4]),
                _rel(got[o + 4:o + 14], ref[o + 4:o + 14]), _rel(got[o + 14:], ref[o + 14:])]
        worst = [max(a, b) for a, b in zip(worst, errs)]
    assert worst[0] <= RTOL_LL and worst[1] <= RTOL_G and worst[2] <= 1e-8 and worst[3] <= RTOL_G, worst
    report.record("config 2 fluA production batch (1024 draws / launch, 28 rows vs C port): loglik %.1e "
                  "grads %.1e Q-params %.1e dLdP %.1e" % tuple(worst))


_SYNTH = {}


def _synthetic_case_ref(n_sites):
    """The synthetic workload and its C-port evaluation (OpenMP, cached per
    size: the full-size tests share one)."""
    if n_sites not in _SYNTH:
        from oracle import cpu
        from phylostan_amd import synthetic
        from phylostan_amd.engine import EvalResult
        pd, prm = synthetic.simulate(n_sites=n_sites)
        case = cases.Case("synthetic", pd.tipcodes, pd.weights, pd.peel0, True, "GTR", 4, prm["blens"],
                          prm["freqs"], prm["rates"], prm["rs"], prm["ps"])
        nt = max(1, min(16, os.cpu_count() or 1))
        out, sl = cpu.evaluate(case.tipcodes, case.weights, case.peel0, True, 2, case.model_vec(), case.blens, 4,
                               site_ll=True, nthreads=nt)
        _SYNTH.clear()
        _SYNTH[n_sites] = (case, EvalResult(out, 2 * case.S - 2, 4, sl))
    return _SYNTH[n_sites]


def _synthetic_vs_c_port(n_sites, engine, devices=None):
    case, ref = _synthetic_case_ref(n_sites)
    eng = _engine(case, devices=devices)
    eng.set_engine(engine)
    res = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    refd = {"site_ll": ref.site_ll, "loglik": ref.loglik, "dLdP": ref.dLdP, "grad_blens": ref.grad_blens,
            "grad_rs": ref.grad_rs, "grad_ps": ref.grad_ps, "grad_freq_root": ref.grad_freq_root}
    e = errors(res, refd, "GTR")
    eq = max(_rel(res.grad_rates, ref.grad_rates), _rel(res.grad_freqs, ref.grad_freqs))
    check(e, eq)
    return case, eng, e, eq


@pytest.mark.parametrize("engine", ["class", "pattern"])
def test_synthetic_full_size_vs_c_port(engine):
    """BASELINE config 4 at full size: 128 taxa x 1,000,000 simulated sites
    (528,111 patterns), GTR+W4 at the simulation's parameters, both engines,
    against the OpenMP C port."""
    case, eng, e, eq = _synthetic_vs_c_port(1_000_000, engine)
    assert case.P == 528111
    if engine == "pattern":
        assert eng.program_info()["nblocks"] > 4000 and eng.lds_plan()["n_chunks"] > 1
    report.record("config 4 synthetic 128x1M (P=%d) [%s] vs C port: %s  Q-params %.1e"
                  % (case.P, engine, fmt(e), eq))


def test_synthetic_full_size_8_shards_vs_c_port():
    """BASELINE config 4's 8-way partition behind ONE handle: phy_create_multi
    over 8 pattern shards of the full 1M-site workload (the one-GPU box maps
    them all to device 0: each shard its own context, class plan and stream,
    rows summed on the device in shard order; on a node with 8 GPUs the same
    handle puts them on devices 0..7 and reduces with one ncclAllReduce)."""
    case, eng, e, eq = _synthetic_vs_c_port(1_000_000, "auto", devices=[0] * 8)
    assert eng.engine() == "class"
    report.record("config 4 synthetic 128x1M in 8 pattern shards (phy_create_multi, P=%d) vs C port: %s  "
                  "Q-params %.1e" % (case.P, fmt(e), eq))


def test_class_sweep_synthetic_200k_vs_c_port():
    """The synthetic workload at 200k sites: the automatic engine choice is
    the class sweep."""
    case, eng, e, eq = _synthetic_vs_c_port(200_000, "auto")
    assert eng.engine() == "class"
    report.record("config 4 synthetic 128x200k (P=%d) [auto=class] vs C port: %s" % (case.P, fmt(e)))


def test_fluA_nuts_config5_full():
    """BASELINE config 5: full NUTS on fluA (4 chains x (1000 warmup + 1000
    draws), seed 1, every leapfrog gradient from the GPU engine); the
    posterior means land inside the 95% intervals the reference prints
    (README.md:104-108)."""
    import time
    from phylostan_amd.engine import TreeLikelihood
    from phylostan_amd.nuts import run_chains
    from tests.test_gpu_inference import README_CI, _fluA_posterior
    post, d = _fluA_posterior(TreeLikelihood, max_draws=4)
    S = d["tipbits"].shape[0]
    q0s = [post.initial_point(np.random.default_rng((1, c))) for c in range(4)]
    t0 = time.perf_counter()
    chains = run_chains(post, q0s, [(1, c) for c in range(4)], num_warmup=1000, num_samples=1000,
                        progress=lambda s: print(s, flush=True))
    wall = time.perf_counter() - t0
    names = post.column_names()
    col = {n: k for k, n in enumerate(names)}
    X = np.concatenate([post.flat_rows(np.stack([dr[0] for dr in ch.draws]))[[not dr[8] for dr in ch.draws]]
                        for ch in chains])
    assert X.shape[0] == 4000
    means = {}
    for key, nm in [("wshape", "wshape"), ("rate", "rate"), ("theta", "theta"), ("kappa", "kappa"),
                    ("root_height", "heights.%d" % (S - 1))]:
        m = float(X[:, col[nm]].mean())
        means[key] = m
        lo, hi = README_CI[key]
        assert lo <= m <= hi, "%s posterior mean %g outside the reference's 95%% CI (%g, %g)" % (key, m, lo, hi)
    report.record("config 5 fluA NUTS 4x(1000+1000) in %.1f s: posterior means inside README CIs: %s"
                  % (wall, ", ".join("%s %.4g" % kv for kv in means.items())))


ZERO_RATE_IDS = ["fluA_HKY_I_W4", "HCV_GTR_I_W4", "HCV_GTR_I", "fluA_HKY_discrete"]


@pytest.mark.parametrize("k", range(4), ids=ZERO_RATE_IDS)
def test_zero_rate_categories_vs_reference(k):
    """A zero-rate category on the device: -I with Weibull
    (generate_script.py:250-266: rs[0] = 0, ps[0] = pinv; t = 0, so P = I and
    the Q-parameter chain rule's Phi takes its tie branch t e^{lambda t} = 0),
    -I with one category (:1231-1240, C = 2) and discrete heterogeneity
    (:1221-1230, free ps).  Every engine -- the quad sweep (a sampler's call),
    the column sweep at one and two columns per lane, the class sweep, and a
    32-draw device-path batch -- against the reference's scripts/phylo.py
    (per-pattern and total log L, rel 1e-10), the oracle (every gradient, rel
    1e-9; the exchangeability / frequency gradients 1e-8) and the reference's
    finite differences of d/drs, d/dps, d/dblens and d/dpinv (rel 1e-6,
    tests/golden/phylo_zero_rate.json)."""
    pt = cases.load_zero_rate_points()[k]
    case = cases.zero_rate_case(pt)
    ref = case.oracle()
    worst = {}
    for engine, cols in (("quad", 0), ("pattern", 1), ("pattern", 2), ("class", 0)):
        eng = _engine(case)
        eng.set_engine("class" if engine == "class" else "pattern")
        if cols:
            eng.set_tuning(cols=cols)
        res = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
        e = errors(res, ref, case.model)
        eq = q_param_error(case, res, ref)
        check(e, eq)
        e_site = _site_rel(res.site_ll, pt["site_ll"])
        e_ll = abs(res.loglik - pt["loglik"]) / abs(pt["loglik"])
        assert e_site <= RTOL_LL and e_ll <= RTOL_LL, (engine, e_site, e_ll)
        fd = cases.zero_rate_errors({"grad_rs": res.grad_rs, "grad_ps": res.grad_ps,
                                     "grad_blens": res.grad_blens}, pt)
        assert all(v <= 1e-6 for v in fd.values()), (engine, fd)
        for key, v in list(fd.items()) + [("loglik", e_ll), ("site_ll", e_site), ("dLdP", e["dLdP"]), ("Q", eq)]:
            worst[key] = max(worst.get(key, 0.0), v)
    # a 32-draw batch (the quad sweep since round 6: calls of <= 32 draws), the point in every row
    n = 32
    eng = _engine(case, max_draws=n)
    rows = eng.evaluate_rows(np.repeat(case.blens[None], n, 0), np.repeat(case.model_vec()[None], n, 0))
    single = _engine(case)
    single.set_tuning(cols=1)
    r1 = single.evaluate_rows(case.blens[None], case.model_vec()[None])[0]
    assert np.all(rows == rows[0])
    assert _rel(rows[0], r1) <= 1e-12
    report.record("site-rate variant %s: vs scripts/phylo.py loglik %.1e site_ll %.1e | vs reference FD %s | "
                  "dLdP vs oracle %.1e Q-params %.1e (quad, K=1, K=2, class, 32-draw batch)"
                  % (ZERO_RATE_IDS[k], worst["loglik"], worst["site_ll"],
                     " ".join("%s %.1e" % (kk, worst[kk]) for kk in ("rs", "ps", "blens", "pinv") if kk in worst),
                     worst["dLdP"], worst["Q"]))
