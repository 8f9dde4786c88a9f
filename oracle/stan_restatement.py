"""Literal restatement of the Stan likelihood that phylostan emits.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Every function below mirrors one block of ``phylostan/generate_script.py`` in
the reference, keeping its loop order and its 1-based indexing so a reader can
hold the two side by side.  Plain Python loops -- use on small inputs only.

Data conventions are those of the Stan ``data`` dict that
``phylostan/phylostan.py:181-286`` builds:

* ``tipdata[S][L][4]``   0/1 partials of the S tips over L patterns
* ``weights[L]``         pattern multiplicities
* ``peel[S-1][3]``       1-based rows ``[child1, child2, parent]`` in post-order
* ``pmats[b + (c-1)*bcount]`` (1-based ``b``) -- 4x4 P-matrices
"""
import math

import numpy as np


# --------------------------------------------------------------------------
# Site-rate heterogeneity  (generate_script.py:249-282, :1209-1220)
# --------------------------------------------------------------------------
def weibull_site_rates(wshape, C):
    """``get_weibull(invariant=False)`` -- generate_script.py:267-278.

    rs[i] = (-log(1 - (2(i-1)+1)/(2C)))^(1/wshape), normalised to mean 1;
    ps = rep_vector(1.0/C, C)  (:1210).
    """
    rs = [0.0] * C
    for i in range(1, C + 1):
        rs[i - 1] = math.pow(-math.log(1.0 - (2.0 * (i - 1) + 1.0) / (2.0 * C)), 1.0 / wshape)
    m = sum(rs) / C
    for i in range(C):
        rs[i] /= m
    ps = [1.0 / C] * C
    return np.array(rs), np.array(ps)


def weibull_pinv_site_rates(wshape, pinv, C):
    """``get_weibull(invariant=True)`` -- generate_script.py:250-266.

    Category 1 is the invariant class (rate 0, weight pinv); the remaining
    C-1 categories share 1-pinv and are normalised so the mean rate is 1.
    """
    rs = [0.0] * C
    ps = [0.0] * C
    cat = C - 1
    pvar = 1.0 - pinv
    rs[0] = 0.0
    ps[0] = pinv
    for i in range(2, C + 1):
        rs[i - 1] = math.pow(-math.log(1.0 - (2.0 * (i - 2) + 1.0) / (2.0 * cat)), 1.0 / wshape)
        ps[i - 1] = pvar / cat
    m = sum(rs) * pvar / cat
    for i in range(2, C + 1):
        rs[i - 1] /= m
    return np.array(rs), np.array(ps)


# --------------------------------------------------------------------------
# P-matrices  (generate_script.py:755-892)
# --------------------------------------------------------------------------
def jc69_p_matrices(blens, rs=None):
    """``calculate_jc69_p_matrices`` -- generate_script.py:755-780."""
    bcount = len(blens)
    rs = [1.0] if rs is None else list(rs)
    C = len(rs)
    pmats = np.zeros((bcount * C, 4, 4))
    index = 0
    for c in range(C):
        for b in range(bcount):
            off = 0.25 - 0.25 * math.exp(-blens[b] * rs[c] / 0.75)
            d = 0.25 + 0.75 * math.exp(-blens[b] * rs[c] / 0.75)
            pmats[index][:, :] = off
            for i in range(4):
                pmats[index][i, i] = d
            index += 1
    return pmats


def _reversible_p_matrices(freqs, R, blens, rs):
    """Shared body of ``calculate_hky_p_matrices`` (:783-836) and
    ``calculate_gtr_p_matrices`` (:839-892)."""
    freqs = np.asarray(freqs, dtype=np.float64)
    rs = [1.0] if rs is None else list(rs)
    C = len(rs)
    bcount = len(blens)
    P2 = np.diag(np.sqrt(freqs))
    P2inv = np.diag(1.0 / np.sqrt(freqs))
    Q = R @ np.diag(freqs)
    s = 0.0
    for i in range(4):
        Q[i, i] = 0.0
        Q[i, i] = -np.sum(Q[i, 0:4])
        s -= Q[i, i] * freqs[i]
    Q = Q / s
    A = P2 @ Q @ P2inv
    # Stan: eigenvalues_sym / eigenvectors_sym (ascending, Eigen's
    # SelfAdjointEigenSolver).  numpy.linalg.eigh has the same contract; P is
    # invariant to eigenvector sign/basis choice.
    eigenvalues, eigenvectors = np.linalg.eigh(A)
    m1 = P2inv @ eigenvectors
    m2 = eigenvectors.T @ P2
    pmats = np.zeros((bcount * C, 4, 4))
    index = 0
    # an extreme draw (a branch of ~1e300) overflows e^(lambda t) for the
    # round-off-positive zero eigenvalue: non-finite P, a rejected draw, as
    # Stan's double arithmetic gives
    with np.errstate(over="ignore", invalid="ignore"):
        for c in range(C):
            for b in range(bcount):
                pmats[index] = m1 @ np.diag(np.exp(eigenvalues * blens[b] * rs[c])) @ m2
                index += 1
    return pmats, Q


def hky_rate_matrix(kappa):
    """Symmetric R of ``calculate_hky_p_matrices`` -- generate_script.py:799-802."""
    return np.array([[0.0, 1.0, kappa, 1.0],
                     [1.0, 0.0, 1.0, kappa],
                     [kappa, 1.0, 0.0, 1.0],
                     [1.0, kappa, 1.0, 0.0]])


def gtr_rate_matrix(rates):
    """Symmetric R of ``calculate_gtr_p_matrices`` -- generate_script.py:855-858.
    Order of ``rates``: AC, AG, AT, CG, CT, GT."""
    r = rates
    return np.array([[0.0, r[0], r[1], r[2]],
                     [r[0], 0.0, r[3], r[4]],
                     [r[1], r[3], 0.0, r[5]],
                     [r[2], r[4], r[5], 0.0]])


def hky_p_matrices(freqs, kappa, blens, rs=None):
    """``calculate_hky_p_matrices`` -- generate_script.py:783-836."""
    return _reversible_p_matrices(freqs, hky_rate_matrix(kappa), blens, rs)[0]


def gtr_p_matrices(freqs, rates, blens, rs=None):
    """``calculate_gtr_p_matrices`` -- generate_script.py:839-892."""
    return _reversible_p_matrices(freqs, gtr_rate_matrix(rates), blens, rs)[0]


# --------------------------------------------------------------------------
# Tree likelihood  (generate_script.py:961-1055)
# --------------------------------------------------------------------------
def stan_loglik(tipdata, weights, peel, pmats, freqs, ps=None, clock=True):
    """The model-block likelihood of ``likelihood(mixture, clock)``.

    ``ps is None`` selects the single-category variants (clock :984-997,
    unrooted :1013-1024); otherwise the mixture variants (clock :998-1012,
    unrooted :1025-1040).  Returns ``(target, per_site)`` where ``per_site[i]``
    is the unweighted site log-likelihood that the loop multiplies by
    ``weights[i]``.  Loops are literal: site outer, node, category inner.
    """
    S = len(tipdata)
    L = len(weights)
    freqs = np.asarray(freqs, dtype=np.float64)
    mixture = ps is not None
    C = len(ps) if mixture else 1
    bcount = len(pmats) // C
    # vector[4] partials[C, 2*S, L]  (1-based node index -> index n-1)
    partials = np.zeros((C, 2 * S, L, 4))
    # copy tip data into node probability vector (:962-983)
    for n in range(1, S + 1):
        for i in range(1, L + 1):
            for a in range(4):
                for c in range(C):
                    partials[c, n - 1, i - 1, a] = tipdata[n - 1][i - 1][a]
    target = 0.0
    per_site = np.zeros(L)

    def pm(b, c):  # pmats[b + (c-1)*bcount], 1-based b and c
        return pmats[b - 1 + (c - 1) * bcount]

    for i in range(1, L + 1):
        if clock:
            for n in range(1, S):
                row = peel[n - 1]
                for c in range(1, C + 1):
                    partials[c - 1, row[2] - 1, i - 1] = (
                        (pm(row[0], c) @ partials[c - 1, row[0] - 1, i - 1])
                        * (pm(row[1], c) @ partials[c - 1, row[1] - 1, i - 1]))
        else:
            for n in range(1, S - 1):
                row = peel[n - 1]
                for c in range(1, C + 1):
                    partials[c - 1, row[2] - 1, i - 1] = (
                        (pm(row[0], c) @ partials[c - 1, row[0] - 1, i - 1])
                        * (pm(row[1], c) @ partials[c - 1, row[1] - 1, i - 1]))
            row = peel[S - 2]
            for c in range(1, C + 1):
                # :1019 / :1034 -- the root branch is merged: no P on child 2
                partials[c - 1, row[2] - 1, i - 1] = (
                    (pm(row[0], c) @ partials[c - 1, row[0] - 1, i - 1])
                    * partials[c - 1, row[1] - 1, i - 1])
        root = peel[S - 2][2]
        if mixture:
            probs = np.zeros(C)
            for c in range(1, C + 1):
                probs[c - 1] = ps[c - 1] * np.sum(partials[c - 1, root - 1, i - 1] * freqs)
            site = math.log(np.sum(probs))
        else:
            site = math.log(np.sum(partials[0, root - 1, i - 1] * freqs))
        per_site[i - 1] = site
        target += site * weights[i - 1]
    return target, per_site
