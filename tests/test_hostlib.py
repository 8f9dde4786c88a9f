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
    ref = _posterior(name, **kw)
    ref._nat = None
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
