"""CPU: the native NUTS chains (csrc/nuts_host.cpp) against nuts.py's
generator chains, their specification: the same seeds give bitwise the same
draws, statistics, gradient counts, step sizes and metrics in every
dimension (both dot products are one sequential sum of rounded products),
through warmup windows, divergences, out-of-support positions, thinning and
short warmups.  And the
whole sampling loop in C++ (phn_run: the posterior's native phases, the
likelihood's submit / wait and the chains) against the same chains driven
round by round through Posterior.log_prob_grad."""
import numpy as np
import pytest

from phylostan_amd import nuts

pytestmark = pytest.mark.skipif(nuts.native_available() is None, reason="libphylo_host.so without NUTS chains")


class Gauss:
    """Independent normals (lp, grad); ``trunc``: lp = -inf below it in x0."""

    def __init__(self, sd, trunc=None, nan_grad_below=None):
        self.sd = np.asarray(sd, np.float64)
        self.dim = self.sd.size
        self.trunc, self.nan_below = trunc, nan_grad_below

    def log_prob_grad(self, U):
        U = np.atleast_2d(U)
        lp = -0.5 * ((U / self.sd) ** 2).sum(1)
        G = -U / self.sd ** 2
        if self.trunc is not None:
            lp = np.where(U[:, 0] < self.trunc, -np.inf, lp)
        if self.nan_below is not None:
            G = np.where((U[:, :1] < self.nan_below), np.nan, G)
        return lp, G


def _pair(tgt, n_chains=3, **kw):
    q0s = [np.full(tgt.dim, 0.3 * k) for k in range(n_chains)]
    seeds = [(5, k) for k in range(n_chains)]
    return (nuts.run_chains(tgt, q0s, seeds, native=False, **kw),
            nuts.run_chains(tgt, q0s, seeds, native=True, **kw))


def _assert_same(a, b):
    assert len(a) == len(b)
    for ca, cb in zip(a, b):
        assert isinstance(cb, nuts.NativeChain)
        assert len(ca.draws) == len(cb.draws)
        assert ca.n_grad == cb.n_grad and ca.eps == cb.eps
        np.testing.assert_array_equal(ca.inv_metric, cb.inv_metric)
        for da, db in zip(ca.draws, cb.draws):
            np.testing.assert_array_equal(da[0], db[0])
            assert da[1:] == db[1:]
            assert [type(x) for x in da[1:]] == [type(x) for x in db[1:]]


@pytest.mark.parametrize("name,sd,kw", [
    ("1d", [2.0], dict(num_warmup=300, num_samples=300)),
    ("2d-aniso", [1.0, 30.0], dict(num_warmup=300, num_samples=200)),
    ("5d", [1, 3, 0.1, 10, 0.5], dict(num_warmup=250, num_samples=100)),
    ("12d", list(np.linspace(0.2, 5, 12)), dict(num_warmup=200, num_samples=100)),
    ("stiff-divergent", [1e-3, 1e3], dict(num_warmup=150, num_samples=50, max_depth=6)),
    ("short-warmup-thin", [1.0, 2.0], dict(num_warmup=15, num_samples=20, thin=3)),
    ("no-warmup", [1.0, 2.0, 3.0], dict(num_warmup=0, num_samples=40)),
    ("options", [1.0, 2.0], dict(num_warmup=120, num_samples=30, delta=0.95, stepsize=0.1, max_delta_h=5.0,
                                  init_buffer=10, term_buffer=10, base_window=5)),
])
def test_native_chains_bitwise_equal_to_generators(name, sd, kw):
    a, b = _pair(Gauss(sd), **kw)
    _assert_same(a, b)


def test_native_chains_out_of_support_and_nan_gradients():
    """lp = -inf regions (divergent leaves, rejected steps) and non-finite
    gradients (zeroed) take the same branches."""
    a, b = _pair(Gauss([1.0, 0.5], trunc=-0.4), num_warmup=150, num_samples=150)
    _assert_same(a, b)
    assert sum(d[6] for c in a for d in c.draws) > 0
    a, b = _pair(Gauss([1.0, 0.5], nan_grad_below=-1.5), num_warmup=100, num_samples=100)
    _assert_same(a, b)


def test_native_chains_long_vectors_bitwise():
    """40 and 150 dimensions (fluA's posterior has ~140): both dot products
    are one sequential sum of rounded products (nuts._sdot / nuts_host.cpp
    dot), so the draws stay bitwise equal whatever the BLAS build vectorises."""
    a, b = _pair(Gauss(np.linspace(0.5, 2.0, 40)), n_chains=2, num_warmup=120, num_samples=40)
    _assert_same(a, b)
    a, b = _pair(Gauss(np.linspace(0.1, 3.0, 150)), n_chains=2, num_warmup=60, num_samples=20)
    _assert_same(a, b)


def test_native_chains_sample_the_target():
    """Moments of a 3-d Gaussian from the native sampler alone."""
    sd = np.array([0.5, 2.0, 4.0])
    ch = nuts.run_chains(Gauss(sd), [np.zeros(3), np.ones(3)], [4, 5], num_warmup=500, num_samples=2000,
                         native=True)
    X = np.concatenate([np.stack([d[0] for d in c.draws if not d[8]]) for c in ch])
    np.testing.assert_allclose(X.std(0), sd, rtol=0.1)
    np.testing.assert_allclose(X.mean(0), 0.0, atol=0.15 * sd.max())


def test_native_chains_errors_match():
    tgt = Gauss([1.0, 1.0], trunc=0.5)
    for native in (False, True):
        with pytest.raises(RuntimeError, match="initial point has non-finite log density"):
            nuts.run_chains(tgt, [np.zeros(2)], [1], num_warmup=10, num_samples=10, native=native)
    with pytest.raises(TypeError):
        nuts.run_chains(Gauss([1.0]), [np.zeros(1)], [1], num_warmup=10, num_samples=10, native=True, bogus=1)


class Flat:
    """A flat density: init_stepsize keeps doubling until the step size
    passes 1e7 ("posterior is improper")."""
    dim = 2

    def log_prob_grad(self, U):
        U = np.atleast_2d(U)
        return np.zeros(U.shape[0]), np.zeros_like(U)


def test_native_chains_improper_posterior():
    for native in (False, True):
        with pytest.raises(RuntimeError, match="improper"):
            nuts.run_chains(Flat(), [np.zeros(2)], [1], num_warmup=10, num_samples=10, native=native)


class _RowsLik:
    """A stand-in likelihood in the TreeLikelihood row layout (log L and
    d/dblens of a Gaussian in the branch lengths, zero Q-parameter
    gradients), reachable both ways: evaluate_rows / submit_rows / wait_rows
    (the Python rounds) and native_submit_wait (C callbacks for phn_run)."""

    def __init__(self, B, C):
        import ctypes
        self.B, self.C = B, C
        self.outlen = 1 + B + 2 * C + 14
        self.calls = 0
        self._pending = None
        SUB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)
        WAIT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)

        def sub(ctx, n, bl, mv):
            self._pending = np.ctypeslib.as_array(ctypes.cast(bl, ctypes.POINTER(ctypes.c_double)),
                                                  shape=(n, self.B)).copy()
            return 0

        def wait(ctx, out):
            rows = self.evaluate_rows(self._pending, None)
            dst = np.ctypeslib.as_array(ctypes.cast(out, ctypes.POINTER(ctypes.c_double)), shape=rows.shape)
            dst[...] = rows
            return 0

        self._cb = (SUB(sub), WAIT(wait))  # alive while the sampler runs

    def evaluate_rows(self, blens, mv):
        self.calls += 1
        x = np.asarray(blens) - 0.02
        rows = np.zeros((x.shape[0], self.outlen))
        rows[:, 0] = -0.5 * 2e3 * (x * x).sum(1)
        rows[:, 1:1 + self.B] = -2e3 * x
        return rows

    def submit_rows(self, blens, mv):
        self._pending = np.array(blens)

    def wait_rows(self):
        return self.evaluate_rows(self._pending, None)

    def native_submit_wait(self, n):
        import ctypes
        return (0, ctypes.cast(self._cb[0], ctypes.c_void_p).value, ctypes.cast(self._cb[1], ctypes.c_void_p).value,
                self.outlen)


def _strict_posterior(lik_factory):
    from phylostan_amd.posterior import ModelSpec, Posterior, TreeData
    from tests import cases
    d = cases.load_layout("fluA")
    S = d["tipbits"].shape[0]
    tree = TreeData(S, d["peel"] - 1, d["map"], d["lowers"], float(d["oldest"]))
    spec = ModelSpec(model="HKY", categories=4, clock="strict", estimate_rate=True, coalescent="constant",
                     heterochronous=True)
    lik = lik_factory(2 * S - 2, 4)
    post = Posterior(spec, tree, lik, compact_rows=True)
    if post._fast is None:
        pytest.skip("the strict-clock posterior's native phases are not built")
    return post, lik


def test_native_loop_equals_python_rounds(monkeypatch):
    """phn_run (pre, likelihood callbacks, post and the chains all in C++)
    gives the draws of the same native chains driven round by round through
    Posterior.log_prob_grad, bit for bit, on the strict-clock fluA posterior
    with a stand-in likelihood; and it made no Python likelihood round trip
    of its own beyond the callbacks."""
    post_a, lik_a = _strict_posterior(_RowsLik)
    post_b, lik_b = _strict_posterior(_RowsLik)
    q0s = [post_a.initial_point(np.random.default_rng((1, c))) for c in range(4)]
    kw = dict(num_warmup=60, num_samples=40, native=True)
    monkeypatch.setenv("PHYLO_NUTS_LOOP", "python")
    a = nuts.run_chains(post_a, q0s, [(1, c) for c in range(4)], **kw)
    monkeypatch.delenv("PHYLO_NUTS_LOOP")
    assert nuts._native_loop_args(post_b, 4) is not None
    b = nuts.run_chains(post_b, q0s, [(1, c) for c in range(4)], **kw)
    assert lik_a.calls == lik_b.calls > 0
    for ca, cb in zip(a, b):
        assert ca.n_grad == cb.n_grad and ca.eps == cb.eps
        for da, db in zip(ca.draws, cb.draws):
            np.testing.assert_array_equal(da[0], db[0])
            assert da[1:] == db[1:]


@pytest.mark.parametrize("name,tgt,kw", [
    ("1d", Gauss([2.0]), dict(num_warmup=200, num_samples=200)),
    ("3d", Gauss([1.0, 2.0, 0.5]), dict(num_warmup=150, num_samples=60)),
    ("rejections", Gauss([1.0, 0.5], trunc=-1.5), dict(num_warmup=100, num_samples=60)),
    ("short-thin", Gauss([1.0, 2.0]), dict(num_warmup=15, num_samples=20, thin=3, int_time=1.0)),
    ("options", Gauss([1.0, 2.0]), dict(num_warmup=120, num_samples=30, delta=0.9, stepsize=0.3, int_time=3.0)),
])
def test_native_static_hmc_bitwise_equal_to_generators(name, tgt, kw):
    """Static HMC (nuts.py StaticHMCChain, Stan's adapt_diag_e_static_hmc) on
    the native chains: the same draws, with the integration time in the
    tree-depth slot as a float."""
    q0s = [np.full(tgt.dim, 0.3 * k) for k in range(3)]
    seeds = [(5, k) for k in range(3)]
    a = nuts.run_chains(tgt, q0s, seeds, native=False, algorithm="hmc", **kw)
    b = nuts.run_chains(tgt, q0s, seeds, native=True, algorithm="hmc", **kw)
    _assert_same(a, b)
    assert isinstance(b[0].draws[0][4], float)


def test_native_static_hmc_errors_match():
    tgt = Gauss([1.0, 1.0], trunc=0.5)
    for native in (False, True):
        with pytest.raises(RuntimeError, match="HMC: initial point has non-finite log density"):
            nuts.run_chains(tgt, [np.zeros(2)], [1], num_warmup=10, num_samples=10, native=native, algorithm="hmc")
