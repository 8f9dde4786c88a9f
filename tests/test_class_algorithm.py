"""CPU: the class sweep's algebra (csrc/class_engine.inc, SURVEY.md 8a row
a10) restated in numpy and checked against the oracle.

The reference's column-reuse prototype (pruner/tree.cpp:140-174) skips a node
whose tip states repeat an earlier column's.  The engine makes that exact:
forward once per distinct subtree tip-state tuple ("class"), reverse on upper
partials aggregated per class.  This test runs the same recursion in numpy --
class pairs, primary/secondary child ordering, aggregated reverse,
G_v = sum_k R_v[k] (x) p_v[k] -- and requires the oracle's log-likelihood,
site values and dL/dP to rel 1e-12.  It is the CPU-side pin of the algebra
the GPU kernels implement (tests/test_gpu_class.py pins the kernels).
"""
import numpy as np
import pytest

from oracle import numpy_pruner as npr
from tests import cases


def class_sweep(case):
    S, P, C = case.S, case.P, case.C
    P_, Q = npr.model_matrices(npr.MODEL_IDS[case.model], case.freqs, case.rates, case.blens, case.rs)  # [C,B,4,4]
    peel = case.peel0
    root = int(peel[-1][2])
    merged = None if case.rooted else int(peel[-1][1])
    tipvec = ((np.arange(16)[:, None] >> np.arange(4)) & 1).astype(np.float64)  # code -> 0/1 state vector
    cls, n, kids = {}, {}, {}
    for t in range(S):
        cls[t] = case.tipcodes[t].astype(np.int64)
        n[t] = 16
    for x, y, v in peel:
        key = cls[x] * n[y] + cls[y]
        u, inv = np.unique(key, return_inverse=True)
        cls[v], n[v] = inv, len(u)
        kids[v] = (u // n[y], u % n[y])
    mat = lambda b: np.eye(4)[None].repeat(C, 0) if b == merged else P_[:, b]  # noqa: E731

    def avec(node, k):  # moved partial of a child's classes: [C, len(k), 4]
        if node < S:
            return np.einsum("cij,kj->cki", mat(node), tipvec[k])
        return A[node][:, k]
    A, pv = {}, {}
    for x, y, v in peel:
        kx, ky = kids[v]
        p = avec(x, kx) * avec(y, ky)
        pv[v] = p
        if v != root:
            A[v] = np.einsum("cij,ckj->cki", mat(v), p)
    # root: one class per distinct full tip-code column; weights summed
    W = np.bincount(cls[root], weights=case.weights, minlength=n[root])
    Lc = case.ps[:, None] * np.einsum("j,ckj->ck", case.freqs, pv[root])
    L = Lc.sum(0)
    site = np.log(L)[cls[root]]
    # aggregated reverse: R_root = (w/L) ps_c pi, identity root branch
    R = {root: (W / L)[None, :, None] * case.ps[:, None, None] * case.freqs[None, None, :]}
    G = np.zeros((C, len(case.blens), 4, 4))
    for x, y, v in peel[::-1]:
        kx, ky = kids[v]
        Rv = R.pop(v)
        if v != root and v != merged:
            G[:, v] = np.einsum("cki,ckj->cij", Rv, pv[v])
            Qv = np.einsum("cji,ckj->cki", mat(v), Rv)
        else:
            Qv = Rv
        for ch, kc, other, ko in ((x, kx, y, ky), (y, ky, x, kx)):
            contrib = Qv * avec(other, ko)  # [C, n_v, 4]
            agg = np.zeros((C, n[ch], 4))
            np.add.at(agg, (slice(None), kc), contrib)  # the segmented reduction
            if ch < S:
                G[:, ch] = np.einsum("cki,kj->cij", agg, tipvec[:n[ch]])
            else:
                R[ch] = agg
    return float(np.dot(case.weights, site)), site, G, sum(n[v] for v in A)


@pytest.mark.parametrize("make", [cases.fluA_case, cases.hcv_case, cases.ds1_case,
                                  lambda: cases.random_case(3, S=30, P=400, C=3, model="GTR"),
                                  lambda: cases.random_case(4, S=17, P=257, C=5, model="GTR", rooted=False)],
                         ids=["fluA", "HCV", "DS1", "random30", "unrooted17"])
def test_class_sweep_algebra_matches_oracle(make):
    case = make()
    ll, site, G, nclasses = class_sweep(case)
    ref = case.oracle()
    assert nclasses < (case.S - 2) * case.P  # subtrees repeat
    assert abs(ll - ref["loglik"]) <= 1e-12 * abs(ref["loglik"])
    np.testing.assert_allclose(site, ref["site_ll"], rtol=1e-12)
    np.testing.assert_allclose(G, ref["dLdP"], rtol=1e-10, atol=1e-12 * np.abs(ref["dLdP"]).max())


def test_repeat_fractions_of_the_configs():
    """The measured a10 repeat fractions DESIGN.md quotes (tools/site_repeats.py)."""
    from tools.site_repeats import report
    for make, frac in ((cases.fluA_case, 0.7653), (cases.hcv_case, 0.7850), (cases.ds1_case, 0.6904)):
        c = make()
        r = report(c.name, c.tipcodes, c.weights, c.peel0)
        assert abs(r["forward_repeat_frac"] - frac) < 1e-4
