"""Stan's constraining transforms (unconstrained R^n -> declared support),
their log-Jacobians, and the reverse pass that carries a gradient w.r.t. the
constrained value back to the unconstrained one.

These are the transforms Stan applies to the ``parameters`` block that
``phylostan/generate_script.py:get_model`` emits (``:1212-1418``):

* ``real<lower=L>``                 x = L + exp(u),            log|J| = u
* ``real<lower=0, upper=1>``        x = inv_logit(u),          log|J| = log x + log(1-x)
* ``simplex[K]``  (K-1 free coords) stick-breaking with the centring offset
  ``log(1/(K-k))`` (Stan Math ``simplex_constrain``), log|J| =
  sum_k log(stick_k) + log z_k + log(1-z_k)
* ``real``                          identity

Every transform works on a batch: ``u`` has shape ``[n, size]``.
"""
import numpy as np


def _log1p_exp(x):
    return np.logaddexp(0.0, x)


def _inv_logit(u):
    """Stan Math's inv_logit: 1 / (1 + e^-u) for u >= 0, e^u / (1 + e^u)
    below (overflow-free; 0 and 1 only where e^-|u| underflows against 1, so
    the native host path, csrc/host_model.cpp, decides support alike)."""
    e = np.exp(-np.abs(u))
    return np.where(u >= 0, 1.0, e) / (1.0 + e)


class Transform:
    """Base: ``size`` unconstrained coordinates -> ``shape`` constrained values."""

    size = 1
    shape = ()

    def constrain(self, u):
        """u [n, size] -> (x [n, *shape], logJ [n], state)."""
        raise NotImplementedError

    def backward(self, state, gx, glogj=1.0):
        """d/du of (sum gx * x + glogj * logJ)  -> [n, size]."""
        raise NotImplementedError

    def unconstrain(self, x):
        raise NotImplementedError


class Identity(Transform):
    def __init__(self, n=None):
        self.size = 1 if n is None else n
        self.shape = () if n is None else (n,)

    def constrain(self, u):
        x = u[:, 0] if not self.shape else u.copy()
        return x, np.zeros(u.shape[0]), None

    def backward(self, state, gx, glogj=1.0):
        return np.asarray(gx, np.float64).reshape(-1, self.size).copy()

    def unconstrain(self, x):
        return np.asarray(x, np.float64).reshape(-1, self.size)


class Lower(Transform):
    """``real<lower=L>`` (or a vector of them)."""

    def __init__(self, lower=0.0, n=None):
        self.lower = float(lower)
        self.size = 1 if n is None else n
        self.shape = () if n is None else (n,)

    def constrain(self, u):
        e = np.exp(u)
        x = self.lower + e
        logj = u.sum(axis=1)
        if not self.shape:
            x = x[:, 0]
        return x, logj, e

    def backward(self, state, gx, glogj=1.0):
        e = state
        gx = np.asarray(gx, np.float64).reshape(e.shape)
        return gx * e + np.asarray(glogj, np.float64).reshape(-1, 1)

    def unconstrain(self, x):
        x = np.asarray(x, np.float64).reshape(-1, self.size)
        return np.log(x - self.lower)


class Unit(Transform):
    """``real<lower=0, upper=1>`` (or a vector of them)."""

    def __init__(self, n=None):
        self.size = 1 if n is None else n
        self.shape = () if n is None else (n,)

    def constrain(self, u):
        x = _inv_logit(u)
        logj = (-_log1p_exp(-u) - _log1p_exp(u)).sum(axis=1)
        state = x
        if not self.shape:
            x = x[:, 0]
        return x, logj, state

    def backward(self, state, gx, glogj=1.0):
        x = state
        gx = np.asarray(gx, np.float64).reshape(x.shape)
        # d x/du = x(1-x);  d logJ/du = 1 - 2x
        return gx * x * (1.0 - x) + np.asarray(glogj, np.float64).reshape(-1, 1) * (1.0 - 2.0 * x)

    def unconstrain(self, x):
        x = np.asarray(x, np.float64).reshape(-1, self.size)
        return np.log(x) - np.log1p(-x)


class Simplex(Transform):
    """``simplex[K]``: K-1 unconstrained coordinates (Stan stick-breaking)."""

    def __init__(self, K):
        self.K = int(K)
        self.size = self.K - 1
        self.shape = (self.K,)
        self.offset = np.log(np.arange(self.K - 1, 0, -1, dtype=np.float64))  # log(K-k), k = 1..K-1

    def constrain(self, u):
        n = u.shape[0]
        K = self.K
        x = np.empty((n, K))
        stick = np.ones(n)
        sticks = np.empty((n, K - 1))
        zs = np.empty((n, K - 1))
        logj = np.zeros(n)
        for k in range(K - 1):
            a = u[:, k] - self.offset[k]
            z = _inv_logit(a)
            sticks[:, k] = stick
            zs[:, k] = z
            x[:, k] = stick * z
            logj += np.log(stick) - _log1p_exp(-a) - _log1p_exp(a)
            stick = stick - x[:, k]
        x[:, K - 1] = stick
        return x, logj, (sticks, zs)

    def backward(self, state, gx, glogj=1.0):
        sticks, zs = state
        n = sticks.shape[0]
        K = self.K
        gx = np.asarray(gx, np.float64).reshape(n, K)
        glogj = np.broadcast_to(np.asarray(glogj, np.float64), (n,))
        gu = np.empty((n, K - 1))
        # adjoint of the running stick after step k (stick_{k+1})
        g_stick = gx[:, K - 1].copy()
        for k in range(K - 2, -1, -1):
            s, z = sticks[:, k], zs[:, k]
            # stick_{k+1} = s - x_k = s (1 - z);  x_k = s z
            g_xk = gx[:, k] - g_stick
            g_s = g_stick + g_xk * z + glogj / s
            g_z = g_xk * s
            # logJ term: -log1p_exp(-a) - log1p_exp(a) -> d/da = 1 - 2z
            gu[:, k] = g_z * z * (1.0 - z) + glogj * (1.0 - 2.0 * z)
            g_stick = g_s
        return gu

    def unconstrain(self, x):
        x = np.asarray(x, np.float64).reshape(-1, self.K)
        u = np.empty((x.shape[0], self.K - 1))
        stick = np.ones(x.shape[0])
        for k in range(self.K - 1):
            z = x[:, k] / stick
            u[:, k] = np.log(z) - np.log1p(-z) + self.offset[k]
            stick = stick - x[:, k]
        return u
