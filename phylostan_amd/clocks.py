"""Relaxed clocks and the birth-death prior of the emitted Stan models, with
gradients.

Restatements of what ``phylostan/generate_script.py`` emits for
``--clock`` other than ``strict`` (``get_model`` ``:1262-1336``) and for
``--speciation bd`` (``:1406-1410``):

* ``get_rates_from_deltas``      ``:42-61``   substrates of the MRF clocks
* ``heights_to_blens`` (non-strict) ``:660-679``  blens = substrates * span
* ``heights_to_blens_autocorr``  ``:682-708``  blens = span * mean of the
  branch's and its parent branch's substrates
* ``ace_log`` ``:187-210``, ``acln_log`` ``:103-141``, ``acg_log``
  ``:144-184``, ``aoup_log`` ``:213-246``
* the ``ucln`` / ``uced`` / ``gmrf`` / ``hsmrf`` prior statements
  ``:1269-1321``
* ``birth_death_log`` ``:2-22``

Branch b is the edge above node b (0-based), so ``substrates[map[j,1]]``
(1-based node id) is ``r[:, node]``.  "Parent rate" follows the Stan code:
the rate of the branch's parent node, except that the children of the root
take the rate of the root's first child ``map[2,1]`` (``f`` below), whose own
rate has the ``exponential(1000)`` prior instead.

Quirks kept for parity (the emitted code is the reference):
* ``aoup_log`` centres every non-root-child rate on its OWN rate
  (``rates[map[i,1]]*exp(-beta*deltaT)``, ``:238``), not its parent's.
* ``heights ~ birth_death(map, 1, netDiversificationRate,
  relativeExtinctionRate)`` binds ``a = netDiversificationRate`` and
  ``r = relativeExtinctionRate`` in ``birth_death_log(heights, map, rho, a,
  r)``; the ``map[i,1] == 1`` branch inside it can never run (node 1 is a tip).
* ``--speciation yule`` adds nothing (get_model only handles ``bd``).

Every function is batched over draws (leading axis ``n``).  Terms that are
constant under ``~`` (Stan ``propto``) are left out; ``dropped_constants``
returns them for ``log_prob(propto=False)``.
"""
import math

import numpy as np
from scipy.special import digamma, gammaln

AUTOCORR = ("ace", "acln", "acg", "aoup", "gmrf", "hsmrf")
MRF = ("gmrf", "hsmrf")
UNCORR = ("ucln", "uced")
RELAXED = AUTOCORR + UNCORR
MRF_SCALE = 0.0014  # deltas ~ normal(0, zeta*[gammas*]0.0014)
UCLN_SD_SHAPE, UCLN_SD_RATE = 0.5396, 2.6184
HALF_LOG_2PI = 0.5 * math.log(2.0 * math.pi)


class ClockTree:
    """Pre-order bookkeeping of ``map`` for the relaxed clocks.

    ``map1`` is the 1-based ``[node, parent]`` pre-order table
    (``utils.get_preorder``); row 0 is the root, row 1 its first child."""

    def __init__(self, S, map1):
        m = np.asarray(map1, np.int64) - 1
        self.S = S
        self.B = 2 * S - 2
        self.root = int(m[0, 0])
        self.f = int(m[1, 0])                      # map[2,1]: the root's first child
        rows = m[2:]                               # Stan rows 3..nodeCount
        self.J = rows[:, 0]                        # node (= branch) of each row
        par = rows[:, 1]
        self.at_root = par == self.root
        self.PR = np.where(self.at_root, self.f, par)  # node whose rate is the "parent rate"
        self.internal_J = self.J >= S
        # map rows in pre-order, so a parent's rate is formed before its children's
        self.delta_of = np.arange(len(self.J))     # deltas[i-2] for row i (1-based)


def blens_multiplier(ct, clock, r):
    """Per-branch factor m [n, B] with blens = span * m, and its adjoint map.

    Uncorrelated clocks: m = r.  Autocorrelated ones (heights_to_blens_autocorr):
    m_f = r_f and m_j = (r_j + r_PR(j)) / 2 for the other rows."""
    if clock in UNCORR:
        return r.copy()
    m = np.empty_like(r)
    m[:, ct.f] = r[:, ct.f]
    m[:, ct.J] = 0.5 * (r[:, ct.J] + r[:, ct.PR])
    return m


def blens_multiplier_backward(ct, clock, g_m):
    """d/dr of sum(g_m * m)."""
    if clock in UNCORR:
        return g_m.copy()
    g = np.zeros_like(g_m)
    g[:, ct.f] += g_m[:, ct.f]
    half = 0.5 * g_m[:, ct.J]
    np.add.at(g.T, ct.J, half.T)
    np.add.at(g.T, ct.PR, half.T)
    return g


def rates_from_deltas(ct, deltas, rate):
    """``get_rates_from_deltas``: r_f = rate, r_j = exp(delta_row + log r_PR(j))."""
    n = deltas.shape[0]
    r = np.empty((n, ct.B))
    r[:, ct.f] = rate
    for k in range(len(ct.J)):  # pre-order: r_PR is already set
        r[:, ct.J[k]] = np.exp(deltas[:, ct.delta_of[k]] + np.log(r[:, ct.PR[k]]))
    return r


def rates_from_deltas_backward(ct, r, g_r):
    """(d/ddeltas, d/drate) of sum(g_r * r)."""
    g_r = g_r.copy()
    gd = np.zeros((r.shape[0], len(ct.J)))
    for k in range(len(ct.J) - 1, -1, -1):  # children before parents
        j, p = ct.J[k], ct.PR[k]
        gj = g_r[:, j] * r[:, j]  # dr_j/d(delta) = r_j, dr_j/dr_p = r_j / r_p
        gd[:, ct.delta_of[k]] += gj
        g_r[:, p] += gj / r[:, p]
    return gd, g_r[:, ct.f]


def _acln(ct, r, span, nu):
    L = np.log(r[:, ct.J])
    M = np.log(r[:, ct.PR])
    t = span[:, ct.J]
    v = nu[:, None] * t
    w = L - M + 0.5 * v
    lp = (-L - 0.5 * np.log(v) - w * w / (2.0 * v)).sum(axis=1)
    dL = -1.0 - w / v
    dM = w / v
    dv = -0.5 / v - w / (2.0 * v) + w * w / (2.0 * v * v)
    return lp, dL / r[:, ct.J], dM / r[:, ct.PR], dv * nu[:, None], (dv * t).sum(axis=1)


def _acg(ct, r, span, nu):
    R = r[:, ct.PR]
    y = r[:, ct.J]
    t = span[:, ct.J]
    v = nu[:, None] * t
    al = R * R / v
    be = R / v
    lp = (al * np.log(be) - gammaln(al) + (al - 1.0) * np.log(y) - be * y).sum(axis=1)
    d_al = np.log(be) - digamma(al) + np.log(y)
    d_be = al / be - y
    d_y = (al - 1.0) / y - be
    d_R = d_al * 2.0 * R / v + d_be / v
    d_v = d_al * (-R * R / (v * v)) + d_be * (-R / (v * v))
    return lp, d_y, d_R, d_v * nu[:, None], (d_v * t).sum(axis=1)


def _ace(ct, r):
    R = r[:, ct.PR]
    y = r[:, ct.J]
    lp = (-np.log(R) - y / R).sum(axis=1)
    return lp, -1.0 / R, -1.0 / R + y / (R * R)


def _aoup(ct, r, span, beta, sig):
    y = r[:, ct.J]
    A = np.where(ct.at_root[None, :], r[:, [ct.f]], y)  # the code's centring rate (see module doc)
    dt = span[:, ct.J]
    b = beta[:, None]
    E = np.exp(-b * dt)
    E2 = E * E
    var = sig[:, None] * (1.0 - E2) / (2.0 * b)
    d = y - A * E
    lp = (-0.5 * np.log(var) - d * d / (2.0 * var)).sum(axis=1)
    g_d = -d / var
    g_var = -0.5 / var + d * d / (2.0 * var * var)
    # d(d)/dy: 1 at root children (A = r_f), 1 - E elsewhere (A = y)
    g_y = g_d * np.where(ct.at_root[None, :], 1.0, 1.0 - E)
    g_f = (g_d * np.where(ct.at_root[None, :], -E, 0.0)).sum(axis=1)
    g_dt = g_d * (A * E * b) + g_var * sig[:, None] * E2
    g_beta = (g_d * A * E * dt + g_var * sig[:, None] * (dt * E2 / b - (1.0 - E2) / (2.0 * b * b))).sum(axis=1)
    g_sig = (g_var * (1.0 - E2) / (2.0 * b)).sum(axis=1)
    return lp, g_y, g_f, g_dt, g_beta, g_sig


def clock_prior(ct, clock, vals, r, span):
    """Prior statements of a relaxed clock.

    vals: constrained parameters by name; r [n, B] substrates; span [n, B]
    branch durations (the ``heights[parent] - heights[node]`` of the
    blens loops).  Returns (lp [n], g_r [n, B], g_span [n, B], {name: grad})."""
    n = r.shape[0]
    lp = np.zeros(n)
    g_r = np.zeros_like(r)
    g_span = np.zeros_like(r)
    gh = {}
    if clock in ("ace", "acln", "acg", "aoup"):
        if clock == "ace":
            l, gy, gR = _ace(ct, r)
            lp += l
            np.add.at(g_r.T, ct.J, gy.T)
            np.add.at(g_r.T, ct.PR, gR.T)
        elif clock in ("acln", "acg"):
            nu = vals["nu"]
            l, gy, gR, gt, gnu = (_acln if clock == "acln" else _acg)(ct, r, span, nu)
            lp += l - nu  # nu ~ exponential(1)
            np.add.at(g_r.T, ct.J, gy.T)
            np.add.at(g_r.T, ct.PR, gR.T)
            g_span[:, ct.J] += gt
            gh["nu"] = gnu - 1.0
        else:
            l, gy, gf, gt, gb, gs = _aoup(ct, r, span, vals["beta"], vals["sigma"])
            lp += l
            g_r[:, ct.J] += gy
            g_r[:, ct.f] += gf
            g_span[:, ct.J] += gt
            gh["beta"], gh["sigma"] = gb, gs
        lp -= 1000.0 * r[:, ct.f]  # substrates[map[2,1]] ~ exponential(1000)
        g_r[:, ct.f] -= 1000.0
    elif clock == "ucln":
        m, s = vals["ucln_mean"], vals["ucln_stdev"]
        mu = np.log(m) - 0.5 * s * s
        L = np.log(r)
        z = L - mu[:, None]
        s2 = (s * s)[:, None]
        B = r.shape[1]
        lp += (-L - z * z / (2.0 * s2)).sum(axis=1) - B * np.log(s)
        g_r += (-1.0 - z / s2) / r
        g_mu = (z / s2).sum(axis=1)
        g_s = -B / s + (z * z).sum(axis=1) / (s * s * s) + g_mu * (-s)
        lp += -1000.0 * m + (UCLN_SD_SHAPE - 1.0) * np.log(s) - UCLN_SD_RATE * s
        gh["ucln_mean"] = g_mu / m - 1000.0
        gh["ucln_stdev"] = g_s + (UCLN_SD_SHAPE - 1.0) / s - UCLN_SD_RATE
    elif clock == "uced":
        m = vals["uced_mean"]
        B = r.shape[1]
        lp += -B * np.log(m) - r.sum(axis=1) / m - 1000.0 * m
        g_r -= 1.0 / m[:, None]
        gh["uced_mean"] = -B / m + r.sum(axis=1) / (m * m) - 1000.0
    elif clock in MRF:
        d = vals["deltas"]
        zeta = vals["zeta"]
        sig = zeta[:, None] * MRF_SCALE * (vals["gammas"] if clock == "hsmrf" else 1.0)
        lp += (-np.log(sig) - d * d / (2.0 * sig * sig)).sum(axis=1)
        g_sig = -1.0 / sig + d * d / (sig ** 3)
        gh["deltas"] = -d / (sig * sig)
        gh["zeta"] = (g_sig * sig).sum(axis=1) / zeta - 2.0 * zeta / (1.0 + zeta * zeta)
        lp -= np.log1p(zeta * zeta)  # zeta ~ cauchy(0, 1)
        if clock == "hsmrf":
            gam = vals["gammas"]
            gh["gammas"] = g_sig * sig / gam - 2.0 * gam / (1.0 + gam * gam)
            lp -= np.log1p(gam * gam).sum(axis=1)  # gammas ~ cauchy(0, 1)
        lp -= 1000.0 * vals["rate"]  # rate ~ exponential(1000)
        gh["rate"] = np.full(n, -1000.0)
    else:
        raise ValueError("not a relaxed clock: %r" % clock)
    return lp, g_r, g_span, gh


def birth_death(heights, a, r):
    """``heights ~ birth_death(map, 1, netDiversificationRate,
    relativeExtinctionRate)``: ``birth_death_log`` with rho = 1 over the S-1
    internal heights [n, S-1].  Returns (lp, d/dheights, d/da, d/dr)."""
    S = heights.shape[1] + 1
    node_count = 2 * S - 1
    A = a[:, None]
    Rr = r[:, None]
    e = np.exp(-Rr * heights)
    q = 1.0 - A * e  # rho + ((1 - rho) - a) e^{-r h} at rho = 1
    z = np.log(q)
    lp = (-2.0 * z - Rr * heights).sum(axis=1) + (S - 1) * np.log(r) + node_count * np.log(1.0 - a)
    g_h = -2.0 * (A * Rr * e / q) - Rr
    g_a = (2.0 * e / q).sum(axis=1) - node_count / (1.0 - a)
    g_r = (-2.0 * A * heights * e / q - heights).sum(axis=1) + (S - 1) / r
    return lp, g_h, g_a, g_r


def dropped_constants(clock, B, n_deltas):
    """Constants the ``~`` statements of a relaxed clock drop (propto)."""
    if clock in ("ace", "acln", "acg", "aoup"):
        c = math.log(1000.0)
        if clock == "acln":
            c += -HALF_LOG_2PI * (B - 1)
        if clock == "aoup":
            c += -HALF_LOG_2PI * (B - 1)
        return c
    if clock == "ucln":
        a, b = UCLN_SD_SHAPE, UCLN_SD_RATE
        return -HALF_LOG_2PI * B + math.log(1000.0) + a * math.log(b) - math.lgamma(a)
    if clock == "uced":
        return math.log(1000.0)
    if clock in MRF:
        k = n_deltas + (n_deltas if clock == "hsmrf" else 0)
        return -HALF_LOG_2PI * n_deltas - math.log(math.pi) * (1 + (k - n_deltas)) + math.log(1000.0)
    return 0.0
