"""CPU: the oracle against the reference's golden values and against itself.

* eigen/test_ll_3tax.py known-answer test (fixture kat_3tax.json, generated
  from the reference's own closed form) -- value and gradient;
* the literal Stan-loop restatement vs the vectorised oracle vs the C oracle;
* analytic gradients vs central finite differences;
* HKY / GTR P-matrices vs scipy.linalg.expm (the Stan Math eigen path is
  absent here: parity unpinned by the reference, pinned to expm instead).
"""
import os
import numpy as np
import pytest
import scipy.linalg

from oracle import numpy_pruner as npr
from oracle import stan_restatement as sr
from phylostan_amd import models
from tests import cases


@pytest.mark.parametrize("k", [0, 1])
def test_kat_3tax(k):
    pt = cases.load_kat()["points"][k]
    case = cases.kat_case(pt)
    # literal Stan loop (generate_script.py:984-997) on the same point
    pm = sr.jc69_p_matrices(case.blens)
    tipdata = np.eye(4)[:3][:, None, :]
    target, _ = sr.stan_loglik(tipdata, [1.0], [[1, 2, 4], [4, 3, 5]], pm, [0.25] * 4)
    assert abs(target - pt["loglik"]) < 1e-13
    ref = case.oracle()
    assert abs(ref["loglik"] - pt["loglik"]) < 1e-13
    g = ref["grad_blens"] * 0.75  # d/dt of the unnormalised-Q closed form
    np.testing.assert_allclose(g[[0, 1, 3, 2]], pt["grad_fd"], rtol=2e-7)


def test_kat_c_oracle():
    from oracle import cpu
    pt = cases.load_kat()["points"][1]
    case = cases.kat_case(pt)
    out, _ = cpu.evaluate(case.tipcodes, case.weights, case.peel0, True, 0, case.model_vec(), case.blens, 1)
    assert abs(out[0] - pt["loglik"]) < 1e-13
    np.testing.assert_allclose(out[1:5][[0, 1, 3, 2]] * 0.75, pt["grad_fd"], rtol=2e-7)


def _to_stan(case, sites):
    """Stan data layout (1-based peel, tipdata [S, L, 4]) of a case subset."""
    tip = npr.tip_vectors(case.tipcodes[:, sites])
    peel = (case.peel0 + 1).tolist()
    return tip, case.weights[sites], peel


@pytest.mark.parametrize("make", [cases.fluA_case, cases.hcv_case, cases.ds1_case,
                                  lambda: cases.random_case(3, S=9, P=30, C=3, model="HKY", rooted=False)])
def test_stan_loop_vs_vectorised(make):
    case = make()
    sites = np.arange(min(case.P, 25))
    tip, w, peel = _to_stan(case, sites)
    P4, _ = npr.model_matrices(npr.MODEL_IDS[case.model], case.freqs, case.rates, case.blens, case.rs)
    pm = P4.reshape(-1, 4, 4)  # index c*B + b == Stan pmats[b + (c-1)*bcount]
    ps = case.ps if case.C > 1 else None
    target, per_site = sr.stan_loglik(tip, w, peel, pm, case.freqs, ps, clock=case.rooted)
    ll, site = npr.loglik_only(case.tipcodes[:, sites], w, case.peel0, case.rooted, P4, case.freqs, case.ps)
    np.testing.assert_allclose(per_site, site, rtol=1e-13, atol=1e-14)
    assert abs(target - ll) <= 1e-12 * abs(ll)


def test_stan_p_matrices_match_vectorised():
    rng = np.random.default_rng(0)
    bl = rng.uniform(0.01, 1.0, 7)
    rs, _ = models.weibull_site_rates(0.6, 3)
    f = rng.dirichlet(np.ones(4) * 4)
    r = rng.uniform(0.5, 3, 6)
    a = sr.gtr_p_matrices(f, r, bl, rs).reshape(3, 7, 4, 4)
    b, _ = npr.model_matrices(npr.GTR, f, r, bl, rs)
    np.testing.assert_allclose(a, b, rtol=0, atol=1e-15)
    a = sr.hky_p_matrices(f, 4.2, bl, rs).reshape(3, 7, 4, 4)
    b, _ = npr.model_matrices(npr.HKY, f, models.hky_exchangeabilities(4.2), bl, rs)
    np.testing.assert_allclose(a, b, rtol=0, atol=1e-15)


@pytest.mark.parametrize("model", ["HKY", "GTR"])
def test_eigen_p_matrices_vs_expm(model):
    rng = np.random.default_rng(1)
    f = rng.dirichlet(np.ones(4) * 3)
    r = models.hky_exchangeabilities(5.0) if model == "HKY" else rng.uniform(0.2, 4, 6)
    bl = np.array([1e-4, 0.05, 0.3, 2.0])
    rs = np.array([0.3, 1.7])
    P, Q = npr.model_matrices(npr.MODEL_IDS[model], f, r, bl, rs)
    for c in range(2):
        for b in range(4):
            np.testing.assert_allclose(P[c, b], scipy.linalg.expm(Q * bl[b] * rs[c]), atol=1e-13)
    np.testing.assert_allclose(P.sum(-1), 1.0, atol=1e-13)  # rows of a transition matrix


def test_jc69_matches_expm():
    bl = np.array([0.01, 0.5, 3.0])
    P, Q = npr.model_matrices(npr.JC69, None, None, bl, [1.0])
    for b in range(3):
        np.testing.assert_allclose(P[0, b], scipy.linalg.expm(Q * bl[b]), atol=1e-14)


def test_weibull_rates():
    for a in (0.2, 0.488, 1.0, 3.0):
        for C in (2, 4, 6):
            rs, ps = models.weibull_site_rates(a, C)
            rs2, ps2 = sr.weibull_site_rates(a, C)
            np.testing.assert_allclose(rs, rs2, rtol=1e-14)
            assert abs(np.mean(rs) - 1) < 1e-13 and np.allclose(ps, 1.0 / C)
            h = 1e-6
            fd = (models.weibull_site_rates(a + h, C)[0] - models.weibull_site_rates(a - h, C)[0]) / (2 * h)
            np.testing.assert_allclose(models.weibull_site_rates_dshape(a, C), fd, rtol=1e-6, atol=1e-9)
    rs, ps = models.weibull_pinv_site_rates(0.7, 0.2, 5)
    rs2, ps2 = sr.weibull_pinv_site_rates(0.7, 0.2, 5)
    np.testing.assert_allclose(rs, rs2, rtol=1e-14)
    np.testing.assert_allclose(ps, ps2, rtol=1e-14)
    assert abs(np.dot(rs, ps) - 1.0) < 1e-13


def _fd(f, x, h=1e-6):
    g = np.zeros_like(x)
    for k in range(x.size):
        e = np.zeros_like(x)
        e[k] = h
        g[k] = (f(x + e) - f(x - e)) / (2 * h)
    return g


@pytest.mark.parametrize("seed,model,rooted", [(1, "GTR", True), (2, "HKY", False), (3, "JC69", True)])
def test_gradients_vs_finite_differences(seed, model, rooted):
    case = cases.random_case(seed, S=7, P=25, C=3, model=model, rooted=rooted)
    mid = npr.MODEL_IDS[model]
    ref = case.oracle()

    def ll(bl=case.blens, rs=case.rs, ps=case.ps, f=case.freqs, r=case.rates):
        P, _ = npr.model_matrices(mid, f, r, bl, rs)
        return npr.loglik_only(case.tipcodes, case.weights, case.peel0, rooted, P, f, ps)[0]

    np.testing.assert_allclose(ref["grad_blens"], _fd(lambda x: ll(bl=x), case.blens), rtol=2e-6, atol=1e-6)
    np.testing.assert_allclose(ref["grad_rs"], _fd(lambda x: ll(rs=x), case.rs), rtol=2e-6, atol=1e-6)
    np.testing.assert_allclose(ref["grad_ps"], _fd(lambda x: ll(ps=x), case.ps), rtol=2e-6, atol=1e-6)
    if model != "JC69":
        gr, gf = models.q_param_gradients(ref["dLdP"], case.blens, case.rs, case.freqs, case.rates,
                                          ref["grad_freq_root"])
        np.testing.assert_allclose(gf, _fd(lambda x: ll(f=x), case.freqs), rtol=2e-6, atol=1e-6)
        if model == "GTR":
            np.testing.assert_allclose(gr, _fd(lambda x: ll(r=x), case.rates), rtol=2e-6, atol=1e-6)
        else:
            k = case.rates[1]
            fdk = (ll(r=models.hky_exchangeabilities(k + 1e-6)) - ll(r=models.hky_exchangeabilities(k - 1e-6))) / 2e-6
            assert abs(models.kappa_gradient(gr) - fdk) < 2e-6 * max(1, abs(fdk))


@pytest.mark.parametrize("make", [cases.fluA_case, cases.hcv_case, cases.ds1_case,
                                  lambda: cases.random_case(6, S=40, P=200, C=4, model="JC69", rooted=False,
                                                            caterpillar=True)])
def test_c_oracle_matches_numpy(make):
    from oracle import cpu
    case = make()
    ref = case.oracle()
    out, sl = cpu.evaluate(case.tipcodes, case.weights, case.peel0, case.rooted, npr.MODEL_IDS[case.model],
                           case.model_vec(), case.blens, case.C, site_ll=True, nthreads=2)
    B = len(case.blens)
    og = 1 + B + 2 * case.C + 4 + 10
    np.testing.assert_allclose(sl, ref["site_ll"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(out[og:], ref["dLdP"].ravel(), rtol=1e-8, atol=1e-9 * np.abs(ref["dLdP"]).max())
    np.testing.assert_allclose(out[1:1 + B], ref["grad_blens"], rtol=1e-8, atol=1e-9 * np.abs(ref["grad_blens"]).max())


def test_linearity_over_pattern_shards():
    """Every output is a sum over patterns: shards add up (the all-reduce)."""
    case = cases.random_case(9, S=10, P=90, C=2)
    P, Q = npr.model_matrices(npr.GTR, case.freqs, case.rates, case.blens, case.rs)
    full = npr.prune(case.tipcodes, case.weights, case.peel0, True, P, case.freqs, case.ps)
    a = npr.prune(case.tipcodes[:, :37], case.weights[:37], case.peel0, True, P, case.freqs, case.ps)
    b = npr.prune(case.tipcodes[:, 37:], case.weights[37:], case.peel0, True, P, case.freqs, case.ps)
    assert abs(a["loglik"] + b["loglik"] - full["loglik"]) < 1e-9
    np.testing.assert_allclose(a["dLdP"] + b["dLdP"], full["dLdP"], rtol=1e-12, atol=1e-12)


def test_q_param_gradients_batch_matches_per_draw():
    """The vectorised chain rule (posterior's path) equals the per-draw one."""
    rng = np.random.default_rng(7)
    n, C, B = 3, 4, 15
    G = rng.normal(size=(n, C, B, 4, 4))
    bl = rng.uniform(0.01, 0.5, (n, B))
    rs = rng.uniform(0.2, 2.0, (n, C))
    f = rng.dirichlet(np.full(4, 3.0), n)
    rt = rng.uniform(0.5, 3.0, (n, 6))
    fr = rng.normal(size=(n, 4))
    gr, gf = models.q_param_gradients_batch(G, bl, rs, f, rt, fr)
    for d in range(n):
        a, b = models.q_param_gradients(G[d], bl[d], rs[d], f[d], rt[d], fr[d])
        np.testing.assert_allclose(gr[d], a, rtol=1e-12, atol=1e-12 * np.max(np.abs(a)))
        np.testing.assert_allclose(gf[d], b, rtol=1e-12, atol=1e-12 * np.max(np.abs(b)))


@pytest.mark.parametrize("k", range(4))
def test_oracle_vs_reference_phylo_py(k):
    """HKY / GTR pinned to the reference's own pruner (scripts/phylo.py):
    total and per-pattern log-likelihoods of the oracle (numpy and C) equal
    the values the reference computed on the fluA / HCV trees."""
    from oracle import cpu
    pt = cases.load_phylo_points()[k]
    case = cases.phylo_case(pt)
    ref = case.oracle()
    np.testing.assert_allclose(ref["site_ll"], pt["site_ll"], rtol=1e-10, atol=1e-12)
    assert abs(ref["loglik"] - pt["loglik"]) <= 1e-10 * abs(pt["loglik"])
    out, sl = cpu.evaluate(case.tipcodes, case.weights, case.peel0, True, npr.MODEL_IDS[case.model],
                           case.model_vec(), case.blens, 1, site_ll=True)
    np.testing.assert_allclose(sl, pt["site_ll"], rtol=1e-10, atol=1e-12)
    assert abs(out[0] - pt["loglik"]) <= 1e-10 * abs(pt["loglik"])


@pytest.mark.parametrize("k", range(3), ids=["fluA_HKY_W4", "HCV_GTR_W4", "DS1_JC69_unrooted"])
def test_oracle_vs_reference_mixture_and_unrooted(k):
    """The configs' own variants pinned to the reference's scripts/phylo.py
    (tests/golden/phylo_mixture.json): the C = 4 Weibull mixture of fluA /
    HCV (generate_script.py:998-1011) and DS1's unrooted merged root branch
    (:1013-1023).  Oracle (numpy and C) per-pattern and total log L at rel
    1e-10 (all-gap patterns, log L ~ 0, at abs 1e-12)."""
    from oracle import cpu
    pt = cases.load_mixture_points()[k]
    case = cases.mixture_case(pt)
    ref = case.oracle()
    np.testing.assert_allclose(ref["site_ll"], pt["site_ll"], rtol=1e-10, atol=1e-12)
    assert abs(ref["loglik"] - pt["loglik"]) <= 1e-10 * abs(pt["loglik"])
    out, sl = cpu.evaluate(case.tipcodes, case.weights, case.peel0, case.rooted, npr.MODEL_IDS[case.model],
                           case.model_vec(), case.blens, case.C, site_ll=True)
    np.testing.assert_allclose(sl, pt["site_ll"], rtol=1e-10, atol=1e-12)
    assert abs(out[0] - pt["loglik"]) <= 1e-10 * abs(pt["loglik"])


def reference_grad_points():
    """tests/golden/phylo_grad.json: central differences (Richardson) of the
    reference's own scripts/phylo.py likelihood, the mixture combined as
    generate_script.py:1006-1010 (tests/golden/make_golden.py grad_fixture)."""
    import json
    with open(os.path.join(cases.GOLDEN, "phylo_grad.json")) as fp:
        return json.load(fp)["points"]


def reference_grad_errors(res_like, pt, case):
    """Max relative errors of an evaluation's gradients against the reference
    FD point: res_like has grad_blens, grad_rs, grad_rates, grad_freqs."""
    from phylostan_amd import models
    errs = {}
    gb = np.asarray(res_like["grad_blens"])[pt["branches"]]
    ref = np.asarray(pt["grad_blens"])
    errs["blens"] = float(np.max(np.abs(gb - ref) / np.maximum(np.abs(ref), 1e-3 * np.max(np.abs(ref)))))
    if "grad_kappa" in pt:
        k = models.kappa_gradient(np.asarray(res_like["grad_rates"]))
        errs["kappa"] = abs(k - pt["grad_kappa"]) / abs(pt["grad_kappa"])
    if "grad_rates" in pt:
        r = np.asarray(pt["grad_rates"])
        errs["rates"] = float(np.max(np.abs(np.asarray(res_like["grad_rates"]) - r)) / np.max(np.abs(r)))
    if "grad_freqs" in pt:
        f = np.asarray(pt["grad_freqs"])
        errs["freqs"] = float(np.max(np.abs(np.asarray(res_like["grad_freqs"]) - f)) / np.max(np.abs(f)))
    if "grad_wshape" in pt:
        dr = models.weibull_site_rates_dshape(pt["wshape"], case.C)
        ga = float(np.dot(np.asarray(res_like["grad_rs"]), dr))
        errs["wshape"] = abs(ga - pt["grad_wshape"]) / abs(pt["grad_wshape"])
    return errs


REF_GRAD_RTOL = 1e-6  # finite differences of the reference (Richardson, h/x = 1e-3 / 1e-4)


@pytest.mark.parametrize("k", range(3), ids=["fluA_HKY_W4", "HCV_GTR_W4", "DS1_JC69_unrooted"])
def test_oracle_gradients_vs_reference_fd(k):
    """The oracle's analytic gradients (branch lengths, kappa or the GTR
    exchangeabilities, frequencies, Weibull shape through rs) against central
    differences of the reference's own likelihood (scripts/phylo.py)."""
    from phylostan_amd import models
    pt = reference_grad_points()[k]
    mp = [p for p in cases.load_mixture_points() if p["dataset"] == pt["dataset"]][0]
    case = cases.mixture_case(mp)
    ref = case.oracle()
    assert abs(ref["loglik"] - pt["loglik"]) <= 1e-10 * abs(pt["loglik"])
    gr, gf = models.q_param_gradients(ref["dLdP"], case.blens, case.rs, case.freqs, case.rates,
                                      ref["grad_freq_root"])
    errs = reference_grad_errors({"grad_blens": ref["grad_blens"], "grad_rs": ref["grad_rs"], "grad_rates": gr,
                                  "grad_freqs": gf}, pt, case)
    assert all(v <= REF_GRAD_RTOL for v in errs.values()), errs


@pytest.mark.parametrize("k", range(4), ids=["fluA_HKY_I_W4", "HCV_GTR_I_W4", "HCV_GTR_I", "fluA_HKY_discrete"])
def test_oracle_zero_rate_categories_vs_reference(k):
    """Zero-rate (+I) and free-weight (discrete) categories: the oracle's
    per-pattern / total log L against the reference's scripts/phylo.py at rel
    1e-10, and its d/drs, d/dps, d/dblens and d/dpinv (through rs and ps)
    against the reference's central differences at 1e-6
    (tests/golden/phylo_zero_rate.json); the C port agrees with the oracle."""
    from oracle import cpu
    from phylostan_amd import models
    pt = cases.load_zero_rate_points()[k]
    case = cases.zero_rate_case(pt)
    ref = case.oracle()
    assert abs(ref["loglik"] - pt["loglik"]) <= 1e-10 * abs(pt["loglik"])
    np.testing.assert_allclose(ref["site_ll"], pt["site_ll"], rtol=1e-10)
    errs = cases.zero_rate_errors(ref, pt)
    assert all(v <= REF_GRAD_RTOL for v in errs.values()), errs
    out, _ = cpu.evaluate(case.tipcodes, case.weights, case.peel0, True, models.MODEL_IDS[case.model],
                          case.model_vec(), case.blens, case.C)
    assert abs(out[0] - ref["loglik"]) <= 1e-12 * abs(ref["loglik"])
