"""NUTS and mean-field ADVI (phylostan_amd/nuts.py, advi.py) on targets with
known answers, and the batched multi-chain driver."""
import math

import numpy as np
import pytest

from phylostan_amd import nuts
from phylostan_amd.advi import ADVI


class Gauss:
    """Independent normal target N(mu, sd^2) with a batched log_prob_grad."""

    def __init__(self, mu, sd):
        self.mu = np.asarray(mu, np.float64)
        self.sd = np.asarray(sd, np.float64)
        self.dim = len(self.mu)
        self.batches = []

    def log_prob_grad(self, Q, propto=True, need_grad=True):
        Q = np.atleast_2d(Q)
        self.batches.append(len(Q))
        z = (Q - self.mu) / self.sd
        lp = -0.5 * (z * z).sum(1)
        if not propto:
            lp = lp - np.log(self.sd).sum() - 0.5 * self.dim * math.log(2 * math.pi)
        return lp, (-(Q - self.mu) / self.sd ** 2 if need_grad else None)

    def log_prob(self, Q, propto=True):
        return self.log_prob_grad(Q, propto, False)[0]


def test_nuts_recovers_gaussian_moments():
    mu = np.array([1.0, -2.0, 0.5, 3.0])
    sd = np.array([0.1, 1.0, 5.0, 0.01])
    tgt = Gauss(mu, sd)
    chains = nuts.run_chains(tgt, [np.zeros(4)], [1], num_warmup=500, num_samples=2000)
    ch = chains[0]
    X = np.stack([d[0] for d in ch.draws if not d[8]])
    assert X.shape == (2000, 4)
    se = sd / math.sqrt(2000) * 4  # generous: autocorrelation
    assert np.all(np.abs(X.mean(0) - mu) < 5 * se)
    np.testing.assert_allclose(X.std(0), sd, rtol=0.15)
    # adapted metric ~ posterior variance, acceptance near delta
    np.testing.assert_allclose(ch.inv_metric, sd ** 2, rtol=0.5)
    acc = np.mean([d[2] for d in ch.draws if not d[8]])
    assert 0.6 < acc < 0.98
    assert all(d[6] == 0 for d in ch.draws if not d[8])


def test_nuts_chains_are_batched():
    tgt = Gauss(np.zeros(3), np.ones(3))
    chains = nuts.run_chains(tgt, [np.full(3, 0.5 * k) for k in range(4)], [10 + k for k in range(4)],
                             num_warmup=50, num_samples=50)
    assert len(chains) == 4 and all(len(c.draws) == 100 for c in chains)
    assert max(tgt.batches) == 4  # one evaluation call serves every pending chain


def test_nuts_window_schedule_matches_stan():
    ch = nuts.Chain(2, np.zeros(2), np.random.default_rng(0), num_warmup=1000)
    ends = []
    for it in range(1000):
        if ch._end_window():
            ends.append(it)
            ch._compute_next_window()
        ch.win_counter += 1
    # Stan: windows 25, 50, 100, 200, 500 after a 75-iteration init buffer, last ends at 949
    assert ends == [99, 149, 249, 449, 949]


def test_advi_meanfield_gaussian():
    mu = np.array([2.0, -1.0, 0.3])
    sd = np.array([0.5, 2.0, 0.05])
    tgt = Gauss(mu, sd)
    adv = ADVI(tgt, np.random.default_rng(3), grad_samples=1, elbo_samples=100, log=None)
    q, eta, iters = adv.run(np.zeros(3), tol_rel_obj=0.001, max_iterations=20000)
    np.testing.assert_allclose(q.mu, mu, atol=3 * sd.max() * 0.2)
    np.testing.assert_allclose(np.exp(q.omega), sd, rtol=0.3)
    # exact ELBO of the optimum for a Gaussian target = 0 (propto=False, KL=0)
    assert abs(adv.calc_elbo(q)) < 0.5
    assert max(tgt.batches) == 100  # the 100 ELBO draws are one batched call


def test_advi_all_eta_fail_is_loud():
    class Bad(Gauss):
        def log_prob_grad(self, Q, propto=True, need_grad=True):
            Q = np.atleast_2d(Q)
            return np.full(len(Q), -np.inf), np.zeros_like(Q)

    with pytest.raises(RuntimeError):
        ADVI(Bad(np.zeros(2), np.ones(2)), np.random.default_rng(0), log=None).run(np.zeros(2))


class CorrGauss:
    """Correlated normal target N(mu, Sigma) with a batched log_prob_grad."""

    def __init__(self, mu, Sigma):
        self.mu = np.asarray(mu, np.float64)
        self.S = np.asarray(Sigma, np.float64)
        self.Si = np.linalg.inv(self.S)
        self.dim = len(self.mu)
        self.batches = []

    def log_prob_grad(self, Q, propto=True, need_grad=True):
        Q = np.atleast_2d(Q)
        self.batches.append(len(Q))
        d = Q - self.mu
        lp = -0.5 * np.einsum("ni,ij,nj->n", d, self.Si, d)
        if not propto:
            lp = lp - 0.5 * np.linalg.slogdet(self.S)[1] - 0.5 * self.dim * math.log(2 * math.pi)
        return lp, (-(d @ self.Si) if need_grad else None)

    def log_prob(self, Q, propto=True):
        return self.log_prob_grad(Q, propto, False)[0]


CORR_MU = np.array([1.5, -0.5, 3.0])
CORR_SIGMA = np.array([[1.0, 0.8, -0.3],
                       [0.8, 2.25, 0.45],
                       [-0.3, 0.45, 0.49]])


def test_advi_fullrank_recovers_correlated_gaussian():
    """normal_fullrank (Stan's advi<Model, normal_fullrank>): on a correlated
    3-D Gaussian the optimum is the target itself -- mean mu, L L^T = Sigma,
    ELBO 0 with propto=False.  Mean-field cannot represent the correlation
    (its variances shrink to 1 / diag(Sigma^-1)), full-rank does."""
    tgt = CorrGauss(CORR_MU, CORR_SIGMA)
    # 10 gradient draws per step (grad_samples): with 1 the SGA iterate
    # wanders ~20 % around the optimum in scale at this iteration count
    adv = ADVI(tgt, np.random.default_rng(3), grad_samples=10, elbo_samples=200, log=None)
    q, eta, iters = adv.run(np.zeros(3), tol_rel_obj=1e-9, max_iterations=20000, family="fullrank")
    assert iters == 20000
    np.testing.assert_allclose(q.mu, CORR_MU, atol=0.08)
    cov = q.L @ q.L.T
    np.testing.assert_allclose(np.diag(cov), np.diag(CORR_SIGMA), rtol=0.1)
    np.testing.assert_allclose(cov, CORR_SIGMA, atol=0.12)
    corr = cov[0, 1] / math.sqrt(cov[0, 0] * cov[1, 1])
    assert abs(corr - 0.8 / 1.5) < 0.08
    assert abs(adv.calc_elbo(q)) < 0.3
    # mean-field on the same target: marginal variances = 1 / diag(Sigma^-1) < diag(Sigma)
    mf = ADVI(CorrGauss(CORR_MU, CORR_SIGMA), np.random.default_rng(3), grad_samples=10, elbo_samples=200,
              log=None)
    qm, _, _ = mf.run(np.zeros(3), tol_rel_obj=1e-9, max_iterations=20000)
    np.testing.assert_allclose(np.exp(2 * qm.omega), 1.0 / np.diag(np.linalg.inv(CORR_SIGMA)), rtol=0.3)


def test_advi_fullrank_gradient_matches_finite_differences():
    """FullRank.grad = d ELBO / d(mu, L) for fixed eta draws: the Monte-Carlo
    ELBO with common random numbers, differentiated numerically."""
    from phylostan_amd.advi import FullRank
    tgt = CorrGauss(CORR_MU, CORR_SIGMA)
    rng = np.random.default_rng(2)
    q = FullRank(np.array([0.3, -0.2, 1.0]), np.array([[1.1, 0, 0], [0.2, 0.7, 0], [-0.1, 0.3, 0.9]]))
    eta = rng.standard_normal((5, 3))

    def elbo(mu, L):
        qq = FullRank(mu, L)
        return float(tgt.log_prob(qq.transform(eta)).mean()) + qq.entropy()

    G = tgt.log_prob_grad(q.transform(eta))[1]
    gmu, gL = q.grad(G, eta)
    h = 1e-6
    for i in range(3):
        e = np.zeros(3)
        e[i] = h
        assert abs((elbo(q.mu + e, q.L) - elbo(q.mu - e, q.L)) / (2 * h) - gmu[i]) < 1e-6
        for j in range(i + 1):
            E = np.zeros((3, 3))
            E[i, j] = h
            assert abs((elbo(q.mu, q.L + E) - elbo(q.mu, q.L - E)) / (2 * h) - gL[i, j]) < 1e-6


def test_static_hmc_recovers_gaussian_moments():
    """Static HMC (sm.sampling(algorithm='HMC'), adapt_diag_e_static_hmc):
    means, standard deviations and the correlation of a correlated Gaussian."""
    tgt = CorrGauss(CORR_MU, CORR_SIGMA)
    # static HMC mixes slowly along the correlated direction (fixed integration
    # time, diagonal metric): 2 x 6000 draws keep the correlation's Monte Carlo
    # error well inside the tolerance (2 x 2000 left it at ~0.05)
    chains = nuts.run_chains(tgt, [np.zeros(3), np.ones(3)], [4, 5], num_warmup=500, num_samples=6000,
                             algorithm="hmc")
    X = np.concatenate([np.stack([d[0] for d in ch.draws if not d[8]]) for ch in chains])
    assert X.shape == (12000, 3)
    sd = np.sqrt(np.diag(CORR_SIGMA))
    assert np.all(np.abs(X.mean(0) - CORR_MU) < 0.1 * sd)
    np.testing.assert_allclose(X.std(0), sd, rtol=0.1)
    c = np.corrcoef(X.T)[0, 1]
    assert abs(c - 0.8 / 1.5) < 0.08
    acc = np.mean([d[2] for ch in chains for d in ch.draws if not d[8]])
    assert 0.5 < acc <= 1.0
    # the sampling phase keeps the last warmup L (no update_L_ in disengage_adaptation)
    for ch in chains:
        n_lf = {d[5] for d in ch.draws if not d[8]}
        assert len(n_lf) == 1


def test_static_hmc_accept_no_overflow():
    """An energy drop of more than ~709 nats over one trajectory (a far-out
    start) is accepted with probability 1, not an OverflowError."""
    tgt = Gauss(np.zeros(2), np.full(2, 0.01))
    with np.errstate(over="ignore"):  # the target's own lp overflows to -inf on the far-out trajectories
        chains = nuts.run_chains(tgt, [np.full(2, 30.0)], [7], num_warmup=30, num_samples=5, algorithm="hmc")
    assert len(chains[0].draws) == 35
