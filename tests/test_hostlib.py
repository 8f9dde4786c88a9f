"""CPU: the native host routines (csrc/host_model.cpp via hostlib) against
their numpy specification in posterior.py / priors.py."""
import numpy as np
import pytest

from phylostan_amd import hostlib, priors
from phylostan_amd.engine import EvalResult
from phylostan_amd.posterior import ModelSpec, Posterior, TreeData
from tests import cases

pytestmark = pytest.mark.skipif(hostlib.load() is None, reason="libphylo_host.so not built")


class SmoothLik:
    """A fast smooth stand-in for the GPU likelihood (host-path tests only)."""

    def __init__(self, B, C):
        self.B, self.C = B, C
        self.outlen = 1 + B + 2 * C + 14

    def evaluate_batch(self, blens, mv, site_ll=False):
        out = []
        for b, m in zip(blens, mv):
            v = np.zeros(self.outlen)
            lb = np.log(b)
            v[0] = -0.5 * np.sum((lb + 3.0) ** 2) + np.sum(np.log(m[10:10 + self.C]))
            v[1:1 + self.B] = -(lb + 3.0) / b
            v[1 + self.B:1 + self.B + self.C] = 1.0 / m[10:10 + self.C]
            out.append(EvalResult(v, self.B, self.C))
        return out


def _posterior(name, **kw):
    d = cases.load_layout(name)
    S = d["tipbits"].shape[0]
    lowers = d.get("lowers")
    oldest = float(d["oldest"]) if "oldest" in d else None
    tree = TreeData(S, d["peel"] - 1, d["map"], lowers, oldest)
    spec = ModelSpec(**kw)
    return Posterior(spec, tree, SmoothLik(2 * S - 2, spec.C))


@pytest.mark.parametrize("name,kw", [
    ("fluA", dict(model="HKY", categories=4, clock="strict", estimate_rate=True, coalescent="constant",
                  heterochronous=True)),
    ("HCV", dict(model="GTR", categories=4, clock="strict", estimate_rate=False, coalescent="constant",
                 heterochronous=False)),
])
def test_native_posterior_equals_numpy(name, kw):
    post = _posterior(name, **kw)
    assert post._nat is not None
    post._fast = None  # the native loops inside the numpy path
    ref = _posterior(name, **kw)
    ref._nat = None
    ref._fast = None
    rng = np.random.default_rng(3)
    U = np.stack([post.initial_point(rng) for _ in range(5)])
    lp_n, g_n = post.log_prob_grad(U)
    lp_r, g_r = ref.log_prob_grad(U)
    np.testing.assert_allclose(lp_n, lp_r, rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(g_n, g_r, rtol=1e-10, atol=1e-9 * np.abs(g_r).max())
    # the same values through the separate transformed-parameters path
    vals, _, _ = post.constrain(U)
    np.testing.assert_allclose(post._heights(vals, 5), ref._heights(vals, 5), rtol=1e-14)


def test_native_constant_coalescent_equals_numpy():
    rng = np.random.default_rng(0)
    n, S = 6, 20
    N = 2 * S - 1
    internal = np.zeros(N, bool)
    internal[S:] = True
    times = np.concatenate([np.round(rng.uniform(0, 2, (n, S)), 1), rng.uniform(1, 5, (n, S - 1))], axis=1)
    times[:, :3] = 0.0  # tied sampling ages
    theta = rng.uniform(0.5, 3.0, n)
    a = hostlib.constant_coalescent(times, internal, theta)
    b = priors.constant_coalescent(times, internal, theta)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-12, atol=1e-12)


class RowsLik:
    """Deterministic compact output rows from (blens, model vectors), every
    entry non-zero -- the Q-parameter and site-rate gradients included."""

    def __init__(self, B, C):
        self.B, self.C = B, C
        self.calls = 0

    def evaluate_rows(self, blens, mv):
        self.calls += 1
        B, C = self.B, self.C
        o = 1 + B + 2 * C
        rows = np.empty((blens.shape[0], o + 14))
        lb = np.log(blens)
        rows[:, 0] = -0.5 * np.sum((lb + 3.0) ** 2, axis=1) + np.log(mv[:, 10:10 + C]).sum(axis=1)
        rows[:, 1:1 + B] = -(lb + 3.0) / blens
        rows[:, 1 + B:o] = np.cos(mv[:, 10:10 + 2 * C]) + 0.5
        rows[:, o:o + 4] = np.sin(mv[:, :4]) * 3.0
        rows[:, o + 4:o + 10] = np.cos(3.0 * mv[:, 4:10])
        rows[:, o + 10:o + 14] = np.sin(2.0 * mv[:, :4]) - 0.25
        return rows


FAST_SPECS = [
    ("fluA", dict(model="HKY", categories=4, clock="strict", estimate_rate=True, coalescent="constant",
                  heterochronous=True)),  # config 5, phylostan's default build
    ("fluA", dict(model="GTR", categories=1, clock="strict", estimate_rate=False, rate=0.004, heterochronous=True)),
    ("HCV", dict(model="JC69", categories=3, clock="strict", estimate_rate=True, coalescent="constant")),
    ("HCV", dict(model="GTR", categories=4, clock="strict", estimate_rate=False, coalescent="constant",
                 speciation="yule")),
]


@pytest.mark.parametrize("name,kw", FAST_SPECS, ids=["fluA_HKY4_rate_const_het", "fluA_GTR1_fixed",
                                                     "HCV_JC3_rate_const", "HCV_GTR4_fixed_const_yule"])
def test_native_strict_posterior_equals_numpy(name, kw):
    """hostlib.StrictPosterior (both phases native) against the numpy
    specification: log density (propto and not) and gradient, including
    out-of-support and non-finite draws (lp = -inf, zero gradient)."""
    def make():
        d = cases.load_layout(name)
        S = d["tipbits"].shape[0]
        tree = TreeData(S, d["peel"] - 1, d["map"], d.get("lowers"), float(d["oldest"]) if "oldest" in d else None)
        spec = ModelSpec(**kw)
        return Posterior(spec, tree, RowsLik(2 * S - 2, spec.C))
    post, ref = make(), make()
    assert post._fast is not None
    ref._fast = None
    rng = np.random.default_rng(11)
    U = np.stack([post.initial_point(rng) for _ in range(7)])
    U[2, post.param("props").sl.start + 3] = 40.0   # props -> 1.0 exactly: out of support
    U[4, post.param("height").sl.start] = np.nan    # non-finite
    U[5] *= 0.1
    for propto in (True, False):
        lp_n, g_n = post.log_prob_grad(U, propto=propto)
        lp_r, g_r = ref.log_prob_grad(U, propto=propto)
        assert np.array_equal(np.isfinite(lp_n), np.isfinite(lp_r))
        assert not np.isfinite(lp_n[2]) and not np.isfinite(lp_n[4])
        fin = np.isfinite(lp_r)
        np.testing.assert_allclose(lp_n[fin], lp_r[fin], rtol=1e-12)
        np.testing.assert_allclose(g_n, g_r, rtol=1e-10, atol=1e-10 * np.abs(g_r).max())
        assert not np.any(g_n[~fin])
    lp_n, g_n = post.log_prob_grad(U, need_grad=False)
    assert g_n is None and np.array_equal(np.isfinite(lp_n), np.isfinite(lp_r))
    # the asynchronous pair (submit / wait) takes the same path
    tok = post.log_prob_grad_begin(U)
    lp_a, g_a = post.log_prob_grad_end(tok)
    np.testing.assert_array_equal(lp_a, post.log_prob_grad(U)[0])


def test_native_strict_posterior_not_used_outside_its_family():
    d = cases.load_layout("fluA")
    S = d["tipbits"].shape[0]
    tree = TreeData(S, d["peel"] - 1, d["map"], d.get("lowers"), float(d["oldest"]))
    for kw in (dict(model="HKY", categories=4, invariant=True, clock="strict", estimate_rate=True),
               dict(model="HKY", categories=4, clock="ucln", estimate_rate=True),
               dict(model="HKY", categories=4, clock="strict", estimate_rate=True, coalescent="skyride"),
               dict(model="HKY", categories=4)):
        spec = ModelSpec(**kw)
        assert Posterior(spec, tree, RowsLik(2 * S - 2, spec.C))._fast is None


def test_native_height_jacobian_tiny_gaps():
    """Nested tiny proportions (early-warmup shapes) on a tree of
    contemporaneous tips: the gaps shrink geometrically down the tree but stay
    positive normal numbers, so the log-Jacobian of the height transform is
    finite; the native product must not underflow where the numpy sum of logs
    does not (host_model.cpp)."""
    kw = dict(model="GTR", categories=4, clock="strict", estimate_rate=False, coalescent="constant",
              heterochronous=False)
    post = _posterior("HCV", **kw)
    assert post._nat is not None
    ref = _posterior("HCV", **kw)
    ref._nat = None
    ref._fast = None
    rng = np.random.default_rng(5)
    us = [-46.0, -20.0, -6.9, -3.0]
    U = np.stack([post.initial_point(rng) for _ in us])
    sl = next(p.sl for p in post.params if p.name == "props")
    for i, u in enumerate(us):
        U[i, sl] = u  # every proportion ~ e^u
    with np.errstate(all="ignore"):
        lp_n, g_n = post.log_prob_grad(U)
        lp_r, g_r = ref.log_prob_grad(U)
    assert np.all(np.isfinite(lp_r))
    np.testing.assert_allclose(lp_n, lp_r, rtol=1e-11)
    np.testing.assert_allclose(g_n, g_r, rtol=1e-9, atol=1e-9 * np.abs(g_r).max())
