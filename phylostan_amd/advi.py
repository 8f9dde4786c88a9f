"""ADVI -- the optimiser behind ``phylostan run -a vb`` (the default;
``phylostan/phylostan.py:302-317``: ``sm.vb(tol_rel_obj, elbo_samples,
grad_samples, iter, eta, algorithm=arg.variational)`` with
``-q meanfield|fullrank``).

Algorithm: Stan's ``advi<Model, normal_meanfield>`` and ``advi<Model,
normal_fullrank>``.  Mean-field: N(mu, diag(exp(omega)^2)) starting at the
initial point with omega = 0.  Full-rank: N(mu, L L^T) with L lower
triangular, starting at L = I; zeta = mu + L eta, entropy
dim/2 (1 + log 2 pi) + sum log|L_dd|, gradient wrt L the lower triangle of
mean(g eta^T) plus 1/L_dd on the diagonal.  Both:
``adapt_eta`` tries eta in (100, 10, 1, 0.1, 0.01) for ``adapt_iter`` (50)
steps each; ``stochastic_gradient_ascent`` uses the adaGrad-like sequence
(history 0.9 / 0.1, tau 1, eta / sqrt(iter)); every ``eval_elbo`` (100)
iterations the ELBO is estimated with ``elbo_samples`` draws and the
relative ELBO change goes into a circular buffer of
max(0.1 max_iter / eval_elbo, 2) entries whose mean or median below
``tol_rel_obj`` stops the run.  The ELBO uses ``log_prob<propto=false>``
(constants included), the gradient ``log_prob<propto=true>``; the entropy
is ``dim/2 (1 + log 2 pi) + sum omega``.  Failed evaluations follow Stan:
``calc_ELBO`` drops a non-finite draw without replacing it and still divides
by ``elbo_samples`` (it gives up once ``elbo_samples`` draws were dropped);
``calc_grad`` throws on the first non-finite gradient draw, which eta
adaptation catches (zero gradient for that iteration) and stochastic
gradient ascent does not -- here (documented in ``calc_elbo_grad``) a failed
gradient draw is redrawn instead, up to 10 * grad_samples times.

MI355X shape: the ``elbo_samples`` draws of each ELBO estimate (default 100)
are ONE batched likelihood launch, as are the ``grad_samples`` draws of each
gradient.
"""
import math
import time

import numpy as np

ETA_SEQUENCE = (100.0, 10.0, 1.0, 0.1, 0.01)


class ADVIError(RuntimeError):
    pass


class MeanField:
    family = "meanfield"

    def __init__(self, mu, omega=None):
        self.mu = np.asarray(mu, np.float64).copy()
        self.omega = np.zeros_like(self.mu) if omega is None else np.asarray(omega, np.float64).copy()

    def copy(self):
        return MeanField(self.mu, self.omega)

    def entropy(self):
        return 0.5 * len(self.mu) * (1.0 + math.log(2.0 * math.pi)) + float(self.omega.sum())

    def transform(self, eta):
        return self.mu + np.exp(self.omega) * eta

    def sample(self, rng, n):
        return self.transform(rng.standard_normal((n, len(self.mu))))

    def grad(self, G, eta):
        """(d mu, d omega) of the ELBO from gradient draws G at transform(eta)."""
        n = G.shape[0]
        mu_g = G.sum(axis=0) / n
        om_g = (G * eta).sum(axis=0) / n
        return mu_g, om_g * np.exp(self.omega) + 1.0

    def params(self):
        return [self.mu, self.omega]


class FullRank:
    """normal_fullrank: N(mu, L L^T), L lower triangular (Cholesky factor)."""
    family = "fullrank"

    def __init__(self, mu, L=None):
        self.mu = np.asarray(mu, np.float64).copy()
        d = len(self.mu)
        self.L = np.eye(d) if L is None else np.tril(np.asarray(L, np.float64)).copy()

    def copy(self):
        return FullRank(self.mu, self.L)

    def entropy(self):
        return (0.5 * len(self.mu) * (1.0 + math.log(2.0 * math.pi))
                + float(np.log(np.abs(np.diag(self.L))).sum()))

    def transform(self, eta):
        return self.mu + eta @ self.L.T

    def sample(self, rng, n):
        return self.transform(rng.standard_normal((n, len(self.mu))))

    def grad(self, G, eta):
        n = G.shape[0]
        mu_g = G.sum(axis=0) / n
        L_g = np.tril(G.T @ eta) / n
        L_g[np.diag_indices_from(L_g)] += 1.0 / np.diag(self.L)
        return mu_g, L_g

    def params(self):
        return [self.mu, self.L]


FAMILIES = {"meanfield": MeanField, "fullrank": FullRank}


class ADVI:
    def __init__(self, posterior, rng, grad_samples=1, elbo_samples=100, eval_elbo=100, log=print):
        self.post = posterior
        self.rng = rng
        self.grad_samples = int(grad_samples)
        self.elbo_samples = int(elbo_samples)
        self.eval_elbo = int(eval_elbo)
        self.log = log or (lambda *_: None)
        self.n_grad = 0
        self.n_lp = 0

    # ------------------------------------------------------------ estimates
    def calc_elbo(self, q):
        """Monte-Carlo ELBO (Stan ``calc_ELBO``): a draw whose log density is
        not finite is dropped, not replaced; the sum is still divided by
        ``elbo_samples``; ``elbo_samples`` drops end the estimate."""
        Z = q.sample(self.rng, self.elbo_samples)
        lp = self.post.log_prob(Z, propto=False)
        self.n_lp += len(Z)
        ok = np.isfinite(lp)
        if int((~ok).sum()) >= self.elbo_samples:
            raise ADVIError("The number of dropped evaluations has reached its maximum amount (%d)."
                            % self.elbo_samples)
        return float(lp[ok].sum()) / self.elbo_samples + q.entropy()

    def calc_elbo_grad(self, q):
        """Stan ``normal_*::calc_grad``: ``grad_samples`` draws, one batched
        launch.  Deliberate difference: Stan throws on the first draw whose
        gradient is not finite (ending the run during stochastic gradient
        ascent); here such a draw is redrawn, and only ``10 * grad_samples``
        failed draws within one estimate end the run.  Draws whose
        transforms overflow in this fp64 numpy host path are rejected
        (``Posterior.in_support``) where Stan's autodiff may still have
        produced a finite value, and one of them should not end a 30k
        iteration run."""
        dim = len(q.mu)
        got_G, got_eta = [], []
        need, drops = self.grad_samples, 0
        while need > 0:
            eta = self.rng.standard_normal((need, dim))
            Z = q.transform(eta)
            lp, G = self.post.log_prob_grad(Z)
            self.n_grad += need
            ok = np.isfinite(lp) & np.all(np.isfinite(G), axis=1)
            got_G.append(G[ok])
            got_eta.append(eta[ok])
            drops += int((~ok).sum())
            need -= int(ok.sum())
            if drops >= 10 * self.grad_samples:
                raise ADVIError("stan::variational::normal_%s::calc_grad: The number of dropped evaluations "
                                "has reached its maximum amount (%d). Your model may be either severely "
                                "ill-conditioned or misspecified." % (q.family, 10 * self.grad_samples))
        return q.grad(np.concatenate(got_G), np.concatenate(got_eta))

    @staticmethod
    def _step(q, grads, hists, it, eta, first):
        """adaGrad-like update of every variational parameter array,
        elementwise (stochastic_gradient_ascent: history 0.9 / 0.1, tau 1)."""
        es = eta / math.sqrt(it)
        for x, g, h in zip(q.params(), grads, hists):
            # a gradient beyond ~1e154 squares to inf here, as in Stan's
            # Eigen arithmetic; that coordinate's step is then 0
            with np.errstate(over="ignore"):
                if first:
                    h += g * g
                else:
                    h *= 0.9
                    h += 0.1 * g * g
            x += es * g / (1.0 + np.sqrt(h))

    # ------------------------------------------------------------ phases
    def adapt_eta(self, q0, adapt_iter=50):
        try:
            elbo_init = self.calc_elbo(q0)
        except ADVIError:
            raise ADVIError("Cannot compute ELBO using the initial variational distribution.")
        self.log("Begin eta adaptation.")
        elbo_best, eta_best = -math.inf, 0.0
        for k, eta in enumerate(ETA_SEQUENCE):
            q = q0.copy()
            hists = [np.zeros_like(x) for x in q.params()]
            for it in range(1, adapt_iter + 1):
                try:
                    grads = self.calc_elbo_grad(q)
                except ADVIError:
                    grads = [np.zeros_like(x) for x in q.params()]
                self._step(q, grads, hists, it, eta, it == 1)
                m = k * adapt_iter + it
                if m == 1 or m % adapt_iter == 0:
                    self.log("Iteration: %3d / %d [%3d%%]  (Adaptation)"
                             % (m, adapt_iter * len(ETA_SEQUENCE), 100 * m // (adapt_iter * len(ETA_SEQUENCE))))
            try:
                elbo = self.calc_elbo(q)
            except ADVIError:
                elbo = -math.inf
            if not np.isfinite(elbo):
                elbo = -math.inf
            if elbo < elbo_best and elbo_best > elbo_init:
                self.log("Success! Found best value [eta = %g]%s" % (eta_best, " earlier than expected."
                                                                   if k < len(ETA_SEQUENCE) - 1 else "."))
                self.log("")
                return eta_best
            if k < len(ETA_SEQUENCE) - 1:
                elbo_best, eta_best = elbo, eta
            else:
                if elbo > elbo_init:
                    self.log("Success! Found best value [eta = %g]." % eta_best)
                    self.log("")
                    return eta
                raise ADVIError("All proposed step-sizes failed. Your model may be either severely "
                                "ill-conditioned or misspecified.")
        return eta_best

    def sga(self, q, eta, tol_rel_obj, max_iterations, diag=None):
        """stochastic_gradient_ascent; ``diag(iter, seconds, elbo)`` per ELBO
        evaluation (the rows of the .diag file)."""
        hists = [np.zeros_like(x) for x in q.params()]
        cb_size = int(max(0.1 * max_iterations / self.eval_elbo, 2.0))
        cb = []
        elbo, elbo_best = 0.0, -math.inf
        self.log("Begin stochastic gradient ascent.")
        self.log("  iter             ELBO   delta_ELBO_mean   delta_ELBO_med   notes ")
        t0 = time.time()
        it = 0
        while True:
            it += 1
            grads = self.calc_elbo_grad(q)
            self._step(q, grads, hists, it, eta, it == 1)
            done = False
            if it % self.eval_elbo == 0:
                elbo_prev = elbo
                elbo = self.calc_elbo(q)
                elbo_best = max(elbo_best, elbo)
                delta = abs((elbo_prev - elbo) / elbo)
                cb.append(delta)
                if len(cb) > cb_size:
                    cb.pop(0)
                ave = float(np.mean(cb))
                med = float(np.median(cb))
                line = "  %4d  %15.3f  %16.3f  %15.3f" % (it, elbo, ave, med)
                if diag:
                    diag(it, time.time() - t0, elbo)
                if ave < tol_rel_obj:
                    line += "   MEAN ELBO CONVERGED"
                    done = True
                if med < tol_rel_obj:
                    line += "   MEDIAN ELBO CONVERGED"
                    done = True
                if it > 10 * self.eval_elbo and (med > 0.5 or ave > 0.5):
                    line += "   MAY BE DIVERGING... INSPECT ELBO"
                self.log(line)
                if done and abs((elbo_best - elbo) / elbo) > 0.05:
                    self.log("Informational Message: The ELBO at a previous iteration is larger than the ELBO "
                             "upon convergence!")
            if it == max_iterations:
                self.log("Informational Message: The maximum number of iterations is reached! The algorithm "
                         "may not have converged.")
                done = True
            if done:
                return q, it

    def run(self, q0_mu, eta=None, adapt_engaged=True, adapt_iter=50, tol_rel_obj=0.01,
            max_iterations=10000, diag=None, family="meanfield"):
        q0 = FAMILIES[family](q0_mu)
        if adapt_engaged or eta is None:
            eta = self.adapt_eta(q0, adapt_iter)
        q, iters = self.sga(q0.copy(), eta, tol_rel_obj, max_iterations, diag)
        return q, eta, iters
