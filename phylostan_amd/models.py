"""Substitution / site-rate models on the host: the parameter vectors the
kernels consume and the chain rule from dlogL/dP back to model parameters.

* ``weibull_site_rates`` / ``weibull_pinv_site_rates`` restate
  ``get_weibull`` (``phylostan/generate_script.py:249-282``); the mixture
  weights are ``ps = 1/C`` (``:1210``).
* ``model_vector`` packs (freqs, exchangeabilities, rs, ps) in the C-ABI
  layout (``include/phylo_hip.h``).  HKY is GTR with exchangeabilities
  ``(1, kappa, 1, 1, kappa, 1)`` -- the R matrix of ``:799-802``.
* ``q_param_gradients`` turns the kernel's dlogL/dP[c][b] into gradients
  w.r.t. the GTR exchangeabilities (or kappa) and the frequencies, through
  the same symmetric eigendecomposition the P-matrices use
  (``:862-876``): with Q = V diag(lam) V^-1,
  d exp(Qt)/dtheta = V ((V^-1 dQ V) o Phi(t)) V^-1,
  Phi_kl = (e^{lam_k t} - e^{lam_l t}) / (lam_k - lam_l)  (t e^{lam t} if equal),
  so sum_{b,c} <G_bc, dP_bc/dtheta> = <V^-1 dQ V, M>,
  M = sum_bc (V^T G_bc V^-T) o Phi_bc  -- M is computed once per evaluation.
"""
import math

import numpy as np

JC69, HKY, GTR = 0, 1, 2
MODEL_IDS = {"JC69": JC69, "HKY": HKY, "GTR": GTR}
GTR_PAIRS = ((0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3))  # AC AG AT CG CT GT


def weibull_site_rates(wshape, C):
    """rs[i] = (-log(1-(2i-1)/(2C)))^(1/wshape) / mean  (generate_script.py:267-278)."""
    i = np.arange(1, C + 1, dtype=np.float64)
    rs = np.power(-np.log(1.0 - (2.0 * (i - 1) + 1.0) / (2.0 * C)), 1.0 / wshape)
    rs = rs / (rs.sum() / C)
    return rs, np.full(C, 1.0 / C)


def weibull_site_rates_dshape(wshape, C):
    """d rs / d wshape for ``weibull_site_rates``."""
    i = np.arange(1, C + 1, dtype=np.float64)
    x = -np.log(1.0 - (2.0 * (i - 1) + 1.0) / (2.0 * C))
    g = np.power(x, 1.0 / wshape)
    dg = g * np.log(x) * (-1.0 / (wshape * wshape))
    m = g.mean()
    dm = dg.mean()
    return dg / m - g * dm / (m * m)


def weibull_pinv_site_rates(wshape, pinv, C):
    """Invariant class + C-1 Weibull classes (generate_script.py:250-266)."""
    cat = C - 1
    rs = np.zeros(C)
    ps = np.zeros(C)
    ps[0] = pinv
    i = np.arange(2, C + 1, dtype=np.float64)
    rs[1:] = np.power(-np.log(1.0 - (2.0 * (i - 2) + 1.0) / (2.0 * cat)), 1.0 / wshape)
    ps[1:] = (1.0 - pinv) / cat
    m = rs.sum() * (1.0 - pinv) / cat
    rs[1:] /= m
    return rs, ps


def hky_exchangeabilities(kappa):
    return np.array([1.0, kappa, 1.0, 1.0, kappa, 1.0])


def model_vector(freqs, rates, rs, ps):
    """[freqs(4), exchangeabilities(6), rs(C), ps(C)] -- the C-ABI layout."""
    return np.concatenate([np.asarray(freqs, np.float64), np.asarray(rates, np.float64),
                           np.asarray(rs, np.float64), np.asarray(ps, np.float64)])


def rate_matrix(freqs, rates):
    """Normalised Q (generate_script.py:862-868) and its pieces."""
    f = np.asarray(freqs, np.float64)
    R = np.zeros((4, 4))
    for k, (i, j) in enumerate(GTR_PAIRS):
        R[i, j] = R[j, i] = rates[k]
    Qt = R * f[None, :]
    np.fill_diagonal(Qt, 0.0)
    np.fill_diagonal(Qt, -Qt.sum(1))
    s = -np.dot(np.diag(Qt), f)
    return Qt / s, R, Qt, s


def eigen_system(freqs, rates):
    """Q = V diag(lam) V^-1 via the symmetric A = Pi^1/2 Q Pi^-1/2
    (generate_script.py:870-876): V = Pi^-1/2 U, V^-1 = U^T Pi^1/2."""
    Q, R, Qt, s = rate_matrix(freqs, rates)
    sq = np.sqrt(np.asarray(freqs, np.float64))
    A = sq[:, None] * Q / sq[None, :]
    A = 0.5 * (A + A.T)
    lam, U = np.linalg.eigh(A)
    V = U / sq[:, None]
    Vinv = U.T * sq[None, :]
    return Q, lam, V, Vinv, R, Qt, s


def _phi(lam, t):
    """Phi[..., k, l] for times t[...]."""
    t = np.asarray(t)[..., None, None]
    lk = lam[:, None]
    ll = lam[None, :]
    ek = np.exp(lk * t)
    el = np.exp(ll * t)
    d = lk - ll
    same = np.abs(d) < 1e-12 * np.maximum(1.0, np.abs(lk))
    with np.errstate(divide="ignore", invalid="ignore"):
        out = np.where(same, t * ek, (ek - el) / np.where(same, 1.0, d))
    return out


def q_param_gradients(dLdP, blens, rs, freqs, rates, grad_freq_root=None):
    """dlogL / d(exchangeabilities[6], freqs[4]) from dlogL/dP[C, B, 4, 4].

    ``grad_freq_root`` (the kernel's explicit root term) is added to the
    frequency gradient.  Returns ``(grad_rates[6], grad_freqs[4])``.
    """
    Q, lam, V, Vinv, R, Qt, s = eigen_system(freqs, rates)
    t = np.asarray(rs)[:, None] * np.asarray(blens)[None, :]  # [C, B]
    H = np.matmul(np.matmul(V.T, dLdP), Vinv.T)  # V^T G V^-T per (c, b)
    M = (H * _phi(lam, t)).sum(axis=(0, 1))
    f = np.asarray(freqs, np.float64)

    def contract(dQt, ds):
        dQ = (dQt - Q * ds) / s
        return float(np.sum((Vinv @ dQ @ V) * M))

    grad_rates = np.zeros(6)
    for k, (i, j) in enumerate(GTR_PAIRS):
        dQt = np.zeros((4, 4))
        dQt[i, j] = f[j]
        dQt[j, i] = f[i]
        dQt[i, i] = -f[j]
        dQt[j, j] = -f[i]
        grad_rates[k] = contract(dQt, 2.0 * f[i] * f[j])
    grad_freqs = np.zeros(4)
    for m in range(4):
        dQt = np.zeros((4, 4))
        for j in range(4):
            if j != m:
                dQt[j, m] = R[j, m]
                dQt[j, j] -= R[j, m]
        ds = 2.0 * sum(R[m, k] * f[k] for k in range(4) if k != m)
        grad_freqs[m] = contract(dQt, ds)
    if grad_freq_root is not None:
        grad_freqs = grad_freqs + np.asarray(grad_freq_root)
    return grad_rates, grad_freqs


def q_param_gradients_batch(dLdP, blens, rs, freqs, rates, grad_freq_root=None):
    """``q_param_gradients`` for n draws at once (dLdP [n, C, B, 4, 4], blens
    [n, B], rs [n, C], freqs [n, 4], rates [n, 6]) -> (grad_rates [n, 6],
    grad_freqs [n, 4]).  Same algebra, vectorised: with M the eigenbasis
    contraction of G and W = V^-T M V^T, each parameter's gradient is
    (sum(dQt * W) - ds * sum(Q * W)) / s with dQt's few nonzeros written out."""
    f = np.asarray(freqs, np.float64)
    rt = np.asarray(rates, np.float64)
    n = f.shape[0]
    R = np.zeros((n, 4, 4))
    for k, (i, j) in enumerate(GTR_PAIRS):
        R[:, i, j] = R[:, j, i] = rt[:, k]
    Qt = R * f[:, None, :]
    idx = np.arange(4)
    Qt[:, idx, idx] = 0.0
    Qt[:, idx, idx] = -Qt.sum(axis=2)
    s = -np.einsum("nii,ni->n", Qt, f)
    Q = Qt / s[:, None, None]
    sq = np.sqrt(f)
    A = sq[:, :, None] * Q / sq[:, None, :]
    A = 0.5 * (A + np.swapaxes(A, 1, 2))
    lam, U = np.linalg.eigh(A)
    V = U / sq[:, :, None]
    Vinv = np.swapaxes(U, 1, 2) * sq[:, None, :]
    t = np.asarray(rs, np.float64)[:, :, None] * np.asarray(blens, np.float64)[:, None, :]  # [n, C, B]
    VT = np.swapaxes(V, 1, 2)[:, None, None]
    VinvT = np.swapaxes(Vinv, 1, 2)[:, None, None]
    H = np.matmul(np.matmul(VT, np.asarray(dLdP, np.float64)), VinvT)  # V^T G V^-T per (c, b)
    # Phi[k, l] = (e^{lam_k t} - e^{lam_l t}) / (lam_k - lam_l), t e^{lam_k t} on ties;
    # the exponentials depend on k only, so they are taken once per (c, b, k)
    E = np.exp(lam[:, None, None, :] * t[..., None])  # [n, C, B, 4]
    ek = E[..., :, None]
    el = E[..., None, :]
    lk = lam[:, None, None, :, None]
    d = lk - lam[:, None, None, None, :]
    same = np.abs(d) < 1e-12 * np.maximum(1.0, np.abs(lk))
    with np.errstate(divide="ignore", invalid="ignore"):
        phi = np.where(same, t[..., None, None] * ek, (ek - el) / np.where(same, 1.0, d))
    M = (H * phi).sum(axis=(1, 2))  # [n, 4, 4]
    W = np.matmul(np.matmul(np.swapaxes(Vinv, 1, 2), M), np.swapaxes(V, 1, 2))  # sum(dQ*W) = sum((Vinv dQ V)*M)
    qw = (Q * W).sum(axis=(1, 2))
    grad_rates = np.empty((n, 6))
    for k, (i, j) in enumerate(GTR_PAIRS):
        dq = f[:, j] * W[:, i, j] + f[:, i] * W[:, j, i] - f[:, j] * W[:, i, i] - f[:, i] * W[:, j, j]
        ds = 2.0 * f[:, i] * f[:, j]
        grad_rates[:, k] = (dq - ds * qw) / s
    grad_freqs = np.empty((n, 4))
    for m in range(4):
        dq = np.zeros(n)
        ds = np.zeros(n)
        for j in range(4):
            if j != m:
                dq += R[:, j, m] * (W[:, j, m] - W[:, j, j])
                ds += 2.0 * R[:, m, j] * f[:, j]
        grad_freqs[:, m] = (dq - ds * qw) / s
    if grad_freq_root is not None:
        grad_freqs = grad_freqs + np.asarray(grad_freq_root, np.float64)
    return grad_rates, grad_freqs


def kappa_gradient(grad_rates):
    """HKY: kappa enters exchangeabilities AG and CT."""
    return float(grad_rates[1] + grad_rates[4])


def empirical_frequencies(tipcodes, weights):
    """Base frequencies of the unambiguous characters (pattern-weighted)."""
    w = np.asarray(weights, np.float64)
    out = np.zeros(4)
    for k, code in enumerate((1, 2, 4, 8)):
        out[k] = ((np.asarray(tipcodes) == code) * w[None, :]).sum()
    return out / out.sum()


def clock_blens(heights, tip_ages, peel0, S, rate):
    """Strict clock: blens[node] = rate * (h[parent] - h[node])
    (generate_script.py:660-679) for every non-root node, 0-based ids."""
    h = np.concatenate([np.asarray(tip_ages, np.float64), np.asarray(heights, np.float64)])
    B = 2 * S - 2
    bl = np.zeros(B)
    for x, y, v in np.asarray(peel0):
        for ch in (x, y):
            if ch < B:
                bl[ch] = rate * (h[v] - h[ch])
    return bl


def jc69_exchangeabilities():
    return np.ones(6)


def ensure_simplex(x):
    x = np.asarray(x, np.float64)
    if np.any(x <= 0) or not math.isclose(float(x.sum()), 1.0, rel_tol=1e-9):
        raise ValueError("expected a positive simplex")
    return x
