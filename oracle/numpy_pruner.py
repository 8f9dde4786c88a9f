"""Vectorised oracle: pruning log-likelihood and its analytic gradient.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Forward pass: the same post-order recurrence as the emitted Stan loop
(``phylostan/generate_script.py:984-1040``), vectorised over patterns and
categories, in fp64 with no rescaling (as the reference).

Reverse pass: the pre-order ("upper partial") recurrence of the reference's
C++ prototypes -- ``pruner/tree.cpp:228-242`` (``q_child = P_child^T
(q_parent .* P_other p_other)``, root ``q = pi``) and
``eigen/eigen.j2:143-167``.  For each branch ``u`` with parent ``v`` and
sibling ``s``::

    r_u = q_v * (P_s p_s)          # upper partial at the top of branch u
    L   = r_u . (P_u p_u)          # site likelihood, any branch
    dL/dP_u = r_u (x) p_u          # outer product
    q_u = P_u^T r_u

so ``dlogL/dP_{b,c} = sum_i w_i ps_c / L_i  r (x) p``.  The chain rule
through ``dP/dt = Q P`` gives the branch-length and rate gradients (the
``times[i]`` factor of ``eigen.j2:165`` is NOT applied: it would give
t * dlogL/dt).

Conventions (the C-ABI's, ``include/phylo_hip.h``): 0-based node ids equal to
the reference's 1-based ids minus one; tips 0..S-1; a branch is named by the
node below it; ``B = 2S-2`` rooted, ``2S-3`` unrooted (node ``2S-3`` is the
root child whose branch is merged, ``generate_script.py:1019``).
"""
import numpy as np

from .stan_restatement import _reversible_p_matrices, gtr_rate_matrix, hky_rate_matrix

JC69, HKY, GTR = 0, 1, 2
MODEL_IDS = {"JC69": JC69, "HKY": HKY, "GTR": GTR}


def tip_vectors(codes):
    """4-bit state masks (A=1, C=2, G=4, T=8) -> 0/1 partial vectors [..., 4]."""
    codes = np.asarray(codes)
    return ((codes[..., None] >> np.arange(4)) & 1).astype(np.float64)


def jc69_q():
    """Rate matrix whose exponential is the Stan JC69 closed form
    ``0.25 +/- ... exp(-t/0.75)`` (generate_script.py:765-766)."""
    return np.full((4, 4), 1.0 / 3.0) - np.eye(4) * (4.0 / 3.0)


def model_matrices(model, freqs, qrates, blens, rs):
    """P-matrices ``[C, B, 4, 4]`` (index ``[c, b]`` == Stan ``pmats[b + c*B]``)
    and the normalised rate matrix Q for JC69 / HKY / GTR.

    ``qrates``: ignored for JC69, kappa (scalar, ``[kappa]`` or the
    exchangeabilities ``(1, kappa, 1, 1, kappa, 1)``) for HKY, the 6
    GTR exchangeabilities (AC, AG, AT, CG, CT, GT) for GTR.
    """
    blens = np.asarray(blens, dtype=np.float64)
    rs = np.asarray(rs, dtype=np.float64)
    if model == JC69:
        t = rs[:, None] * blens[None, :]
        e = np.exp(-t / 0.75)
        P = np.empty(t.shape + (4, 4))
        P[...] = (0.25 - 0.25 * e)[..., None, None]
        idx = np.arange(4)
        P[..., idx, idx] = (0.25 + 0.75 * e)[..., None]
        return P, jc69_q()
    if model == HKY:
        q = np.ravel(np.asarray(qrates, dtype=np.float64))
        if q.size == 6:  # exchangeability form (1, kappa, 1, 1, kappa, 1)
            if not (np.allclose(q[[0, 2, 3, 5]], 1.0) and q[1] == q[4]):
                raise ValueError("not an HKY exchangeability vector")
            q = q[1:2]
        R = hky_rate_matrix(float(q[0]))
    elif model == GTR:
        R = gtr_rate_matrix(np.asarray(qrates, dtype=np.float64))
    else:
        raise ValueError("model must be JC69, HKY or GTR")
    pm, Q = _reversible_p_matrices(freqs, R, blens, rs)
    return pm.reshape(len(rs), len(blens), 4, 4), Q


def prune(tipcodes, weights, peel, rooted, pmats, freqs, ps, Q=None, blens=None, rs=None):
    # L = 0 (a draw the sampler rejects): log L = -inf and non-finite
    # gradients, as the GPU's -inf row -- not a numerical fault of the oracle
    with np.errstate(divide="ignore", invalid="ignore"):
        return _prune(tipcodes, weights, peel, rooted, pmats, freqs, ps, Q, blens, rs)


def _prune(tipcodes, weights, peel, rooted, pmats, freqs, ps, Q=None, blens=None, rs=None):
    """Log-likelihood and gradient of one parameter point.

    Parameters
    ----------
    tipcodes : uint8 [S, P] state masks
    weights  : float [P]
    peel     : int [S-1, 3] 0-based (child1, child2, parent), post-order
    rooted   : bool -- clock (rooted) or unrooted variant
    pmats    : float [C, B, 4, 4]
    freqs, ps: root frequencies [4], category weights [C]
    Q, blens, rs : optional -- when given, ``grad_blens`` / ``grad_rs`` are
                   added via dP/dt = Q P.

    Returns a dict with ``loglik``, ``site_ll[P]``, ``dLdP[C,B,4,4]``,
    ``grad_ps[C]``, ``grad_freq_root[4]`` and optionally ``grad_blens[B]``,
    ``grad_rs[C]``.
    """
    tipcodes = np.asarray(tipcodes)
    S, P = tipcodes.shape
    peel = np.asarray(peel, dtype=np.int64)
    C, B = pmats.shape[:2]
    freqs = np.asarray(freqs, dtype=np.float64)
    ps = np.asarray(ps, dtype=np.float64)
    w = np.asarray(weights, dtype=np.float64)
    n_nodes = 2 * S - 1
    root = int(peel[-1, 2])
    merged = None if rooted else int(peel[-1, 1])  # child with no branch

    def branch(node):
        return None if node == merged else node

    part = [None] * n_nodes
    for t in range(S):
        part[t] = np.broadcast_to(tip_vectors(tipcodes[t]), (C, P, 4))
    moved = {}
    for x, y, v in peel:
        ax = np.einsum("cjk,cpk->cpj", pmats[:, x], part[x])
        by = branch(y)
        ay = part[y] if by is None else np.einsum("cjk,cpk->cpj", pmats[:, by], part[y])
        moved[x], moved[y] = ax, ay
        part[v] = ax * ay
    Lc = ps[:, None] * np.einsum("j,cpj->cp", freqs, part[root])  # [C, P]
    L = Lc.sum(axis=0)
    site_ll = np.log(L)
    loglik = float(np.dot(w, site_ll))
    sc = w / L  # [P]

    grad_ps = np.einsum("p,cp->c", sc, Lc / ps[:, None])
    grad_freq_root = np.einsum("p,c,cpj->j", sc, ps, part[root])

    s_cp = ps[:, None] * sc[None, :]  # [C, P]
    dLdP = np.zeros((C, B, 4, 4))
    q = [None] * n_nodes
    q[root] = np.broadcast_to(freqs, (C, P, 4))
    for x, y, v in peel[::-1]:
        ax, ay = moved[x], moved[y]
        rx = q[v] * ay
        ry = q[v] * ax
        dLdP[:, x] += np.einsum("cp,cpj,cpk->cjk", s_cp, rx, part[x])
        q[x] = np.einsum("cjk,cpj->cpk", pmats[:, x], rx)
        by = branch(y)
        if by is None:
            q[y] = ry
        else:
            dLdP[:, by] += np.einsum("cp,cpj,cpk->cjk", s_cp, ry, part[y])
            q[y] = np.einsum("cjk,cpj->cpk", pmats[:, by], ry)
    out = dict(loglik=loglik, site_ll=site_ll, dLdP=dLdP, grad_ps=grad_ps,
               grad_freq_root=grad_freq_root)
    if Q is not None:
        QP = np.einsum("jl,cblk->cbjk", Q, pmats)
        inner = np.einsum("cbjk,cbjk->cb", dLdP, QP)  # dlogL/dt_{b,c}
        rs = np.asarray(rs, dtype=np.float64)
        blens = np.asarray(blens, dtype=np.float64)
        out["grad_blens"] = np.einsum("c,cb->b", rs, inner)
        out["grad_rs"] = np.einsum("b,cb->c", blens, inner)
    return out


def loglik_only(tipcodes, weights, peel, rooted, pmats, freqs, ps):
    """Forward pass only (cheap; used for finite differences)."""
    tipcodes = np.asarray(tipcodes)
    S, P = tipcodes.shape
    C = pmats.shape[0]
    root = int(peel[-1][2])
    merged = None if rooted else int(peel[-1][1])
    part = {}
    for t in range(S):
        part[t] = np.broadcast_to(tip_vectors(tipcodes[t]), (C, P, 4))
    for x, y, v in peel:
        ax = np.einsum("cjk,cpk->cpj", pmats[:, x], part[x])
        ay = part[y] if y == merged else np.einsum("cjk,cpk->cpj", pmats[:, y], part[y])
        part[v] = ax * ay
    L = (np.asarray(ps)[:, None] * np.einsum("j,cpj->cp", np.asarray(freqs), part[root])).sum(0)
    with np.errstate(divide="ignore"):  # L = 0: -inf, a rejected draw
        return float(np.dot(weights, np.log(L))), np.log(L)
