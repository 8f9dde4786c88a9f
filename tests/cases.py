"""Shared test cases: golden fixtures, parameter points and random trees.

Parameter points of the configs (BASELINE.json / SURVEY.md 8d):
  fluA  HKY+W4 strict clock: kappa 5.58, wshape 0.488, rate 0.00499,
        input-tree heights, empirical frequencies (README.md:104-108)
  HCV   GTR+W4: rates (1,2,1,1,2,1)/8, freqs 1/4, wshape 0.5, rate 7.9e-4
        (examples/SConstruct:218), input-tree heights
  DS1   JC69 unrooted, blens ~ Exp(10) (generate_script.py:1404), seed 0
"""
import json
import os

import numpy as np

from phylostan_amd import models

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_layout(name):
    z = np.load(os.path.join(GOLDEN, "%s_layout.npz" % name), allow_pickle=False)
    return {k: z[k] for k in z.files}


def load_kat():
    with open(os.path.join(GOLDEN, "kat_3tax.json")) as fp:
        return json.load(fp)


def load_phylo_points():
    """HKY / GTR points evaluated by the reference's scripts/phylo.py
    (tests/golden/make_golden.py, ``phylo_gtr_fixture``)."""
    with open(os.path.join(GOLDEN, "phylo_gtr.json")) as fp:
        return json.load(fp)["points"]


def phylo_case(point):
    """One scripts/phylo.py point as a C = 1 case on the dataset's compressed
    layout (weights = column multiplicities, so sum w l = the reference's sum
    over every alignment column)."""
    d = load_layout(point["dataset"])
    return Case("phylo_%s_%s" % (point["dataset"], point["model"]), d["tipbits"], d["weights"], d["peel"] - 1,
                True, point["model"], 1, point["blens"], point["freqs"], point["rates"], [1.0], [1.0])


def load_mixture_points():
    """The configs' own variants evaluated by the reference's scripts/phylo.py
    (tests/golden/make_golden.py ``mixture_fixture``): fluA HKY+W4 and HCV
    GTR+W4 (C = 4 Weibull mixture) and DS1 JC69 unrooted (merged root edge)."""
    with open(os.path.join(GOLDEN, "phylo_mixture.json")) as fp:
        return json.load(fp)["points"]


def mixture_case(point):
    d = load_layout(point["dataset"])
    S = d["tipbits"].shape[0]
    B = 2 * S - 2 if point["rooted"] else 2 * S - 3
    return Case("ref_%s_%s" % (point["dataset"], point["model"]), d["tipbits"], d["weights"], d["peel"] - 1,
                point["rooted"], point["model"], point["C"], point["blens"][:B], point["freqs"], point["rates"],
                point["rs"], point["ps"])


class Case:
    """One likelihood problem in C-ABI conventions."""

    def __init__(self, name, tipcodes, weights, peel0, rooted, model, C, blens, freqs, rates, rs, ps):
        self.name = name
        self.tipcodes = np.ascontiguousarray(tipcodes, dtype=np.uint8)
        self.weights = np.asarray(weights, dtype=np.float64)
        self.peel0 = np.asarray(peel0, dtype=np.int32)
        self.rooted = rooted
        self.model = model
        self.C = C
        self.blens = np.asarray(blens, dtype=np.float64)
        self.freqs = np.asarray(freqs, dtype=np.float64)
        self.rates = np.asarray(rates, dtype=np.float64)
        self.rs = np.asarray(rs, dtype=np.float64)
        self.ps = np.asarray(ps, dtype=np.float64)

    @property
    def S(self):
        return self.tipcodes.shape[0]

    @property
    def P(self):
        return self.tipcodes.shape[1]

    def model_vec(self):
        return models.model_vector(self.freqs, self.rates, self.rs, self.ps)

    def oracle(self):
        from oracle import numpy_pruner as npr
        P, Q = npr.model_matrices(npr.MODEL_IDS[self.model], self.freqs, self.rates, self.blens, self.rs)
        return npr.prune(self.tipcodes, self.weights, self.peel0, self.rooted, P, self.freqs, self.ps,
                         Q=Q, blens=self.blens, rs=self.rs)


def fluA_case():
    d = load_layout("fluA")
    S = d["tipbits"].shape[0]
    peel0 = d["peel"] - 1
    rate = 0.00499
    blens = models.clock_blens(d["heights"], d["tip_dates"], peel0, S, rate)
    freqs = models.empirical_frequencies(d["tipbits"], d["weights"])
    rs, ps = models.weibull_site_rates(0.488, 4)
    return Case("fluA", d["tipbits"], d["weights"], peel0, True, "HKY", 4, blens, freqs,
                models.hky_exchangeabilities(5.58), rs, ps)


def hcv_case():
    d = load_layout("HCV")
    S = d["tipbits"].shape[0]
    peel0 = d["peel"] - 1
    blens = models.clock_blens(d["heights"], d["tip_dates"], peel0, S, 7.9e-4)
    rates = np.array([1.0, 2.0, 1.0, 1.0, 2.0, 1.0]) / 8.0
    rs, ps = models.weibull_site_rates(0.5, 4)
    return Case("HCV", d["tipbits"], d["weights"], peel0, True, "GTR", 4, blens, np.full(4, 0.25),
                rates, rs, ps)


def ds1_case(seed=0):
    d = load_layout("DS1")
    S = d["tipbits"].shape[0]
    rng = np.random.default_rng(seed)
    blens = rng.exponential(1.0 / 10.0, size=2 * S - 3)
    return Case("DS1", d["tipbits"], d["weights"], d["peel"] - 1, False, "JC69", 1, blens,
                np.full(4, 0.25), np.ones(6), [1.0], [1.0])


def ds1_topology_case(k):
    """Config 1 on DS1 topology k of the 42 in examples/DS1/DS1.trees (the
    reference pipeline's tree{k}.tree, examples/SConstruct:159-188): its
    layout from the reference's utils.py and the blens of its reference
    per-site log-likelihoods (tests/golden/DS1_topologies.npz)."""
    d = np.load(os.path.join(GOLDEN, "DS1_topologies.npz"), allow_pickle=False)
    tip = d["tipbits0"][d["perm"][k]]
    j = int(np.nonzero(d["ll_topologies"] == k)[0][0])
    return Case("DS1_tree%d" % k, tip, d["weights"], d["peel"][k] - 1, False, "JC69", 1, d["blens"][j],
                np.full(4, 0.25), np.ones(6), [1.0], [1.0])


def ds1_topology_reference(k):
    """The reference's (scripts/phylo.py) per-pattern log-likelihoods and total
    for DS1 topology k at ds1_topology_case(k)'s branch lengths."""
    d = np.load(os.path.join(GOLDEN, "DS1_topologies.npz"), allow_pickle=False)
    j = int(np.nonzero(d["ll_topologies"] == k)[0][0])
    return d["site_ll"][j], float(d["loglik"][j])


def kat_case(point):
    """3-taxon KAT of eigen/test_ll_3tax.py in Stan JC69 units (b = 0.75 t)."""
    b14, b24, b45, b35 = point["branches_b14_b24_b45_b35"]
    blens = 0.75 * np.array([b14, b24, b35, b45])  # node ids 0, 1, 2, 3
    return Case("kat", np.array([[1], [2], [4]]), [1.0], [[0, 1, 3], [3, 2, 4]], True, "JC69", 1,
                blens, np.full(4, 0.25), np.ones(6), [1.0], [1.0])


def random_peel(S, rng, caterpillar=False):
    """Random rooted binary topology (0-based ids, post-order indexing like
    utils.setup_indexes: internal nodes numbered in creation order)."""
    if caterpillar:
        peel = [[0, 1, S]]
        for k in range(2, S):
            peel.append([S + k - 2, k, S + k - 1])
        return np.array(peel, dtype=np.int32)
    nodes = list(range(S))
    nxt = S
    peel = []
    while len(nodes) > 1:
        i, j = rng.choice(len(nodes), 2, replace=False)
        a, b = nodes[i], nodes[j]
        for k in sorted((i, j), reverse=True):
            nodes.pop(k)
        peel.append([a, b, nxt])
        nodes.append(nxt)
        nxt += 1
    return np.array(peel, dtype=np.int32)


def make_unrooted(peel):
    """Apply phylostan.py:264-267: the root row's larger child goes second;
    it must be node 2S-3 (the last internal node before the root)."""
    peel = np.array(peel, dtype=np.int32)
    S = peel.shape[0] + 1
    last = peel[-1]
    if last[0] > last[1]:
        peel[-1] = [last[1], last[0], last[2]]
    assert peel[-1][1] == 2 * S - 3, "root child 2 must be node 2S-3"
    return peel


def random_case(seed, S=12, P=100, C=3, model="GTR", rooted=True, caterpillar=False,
                ambiguous=0.1):
    rng = np.random.default_rng(seed)
    peel = random_peel(S, rng, caterpillar)
    if not rooted:
        # make sure the root has an internal second child = node 2S-3
        last = peel[-1]
        if 2 * S - 3 not in (last[0], last[1]):
            return random_case(seed + 1000, S, P, C, model, rooted, caterpillar, ambiguous)
        peel = make_unrooted(peel)
    codes = rng.choice([1, 2, 4, 8], size=(S, P)).astype(np.uint8)
    amb = rng.random((S, P)) < ambiguous
    codes[amb] = rng.choice([15, 3, 5, 10, 6], size=amb.sum())
    w = rng.integers(1, 5, P).astype(np.float64)
    B = 2 * S - 2 if rooted else 2 * S - 3
    blens = rng.uniform(0.01, 0.3, B)
    freqs = rng.dirichlet(np.full(4, 5.0))
    rates = rng.uniform(0.5, 3.0, 6)
    if model == "HKY":
        rates = models.hky_exchangeabilities(rng.uniform(1.0, 8.0))
    if model == "JC69":
        freqs = np.full(4, 0.25)
        rates = np.ones(6)
    rs, ps = models.weibull_site_rates(rng.uniform(0.3, 2.0), C)
    return Case("rand%d" % seed, codes, w, peel, rooted, model, C, blens, freqs, rates, rs, ps)


def load_zero_rate_points():
    """Site-rate variants with a zero-rate or free-weight category (+I with
    Weibull, +I with one category, discrete heterogeneity) evaluated by the
    reference's scripts/phylo.py (tests/golden/make_golden.py
    ``zero_rate_fixture``)."""
    with open(os.path.join(GOLDEN, "phylo_zero_rate.json")) as fp:
        return json.load(fp)["points"]


def zero_rate_case(point):
    d = load_layout(point["dataset"])
    return Case("zr_%s_%s_%s" % (point["dataset"], point["model"], point["kind"]), d["tipbits"], d["weights"],
                d["peel"] - 1, True, point["model"], point["C"], point["blens"], point["freqs"], point["rates"],
                point["rs"], point["ps"])


def zero_rate_dpinv(point):
    """(drs/dpinv, dps/dpinv) of the point's +I site rates
    (generate_script.py:250-266, :1231-1240) by central differences of the
    host restatement (exact to ~1e-10 relative)."""
    from tests.golden.make_golden import _zero_rate_rates
    h = 1e-6
    a = _zero_rate_rates(point["kind"], point["pinv"] + h, point.get("wshape"))
    b = _zero_rate_rates(point["kind"], point["pinv"] - h, point.get("wshape"))
    return (np.asarray(a[0]) - np.asarray(b[0])) / (2 * h), (np.asarray(a[1]) - np.asarray(b[1])) / (2 * h)


def zero_rate_errors(res_like, pt):
    """Max relative errors of an evaluation's site-rate and branch gradients
    against the point's reference finite differences."""
    errs = {}
    for key in ("grad_rs", "grad_ps"):
        ref = np.asarray(pt[key])
        errs[key[5:]] = float(np.max(np.abs(np.asarray(res_like[key]) - ref)) / np.max(np.abs(ref)))
    gb = np.asarray(res_like["grad_blens"])[pt["branches"]]
    ref = np.asarray(pt["grad_blens"])
    errs["blens"] = float(np.max(np.abs(gb - ref)) / np.max(np.abs(ref)))
    if "grad_pinv" in pt:
        drs, dps = zero_rate_dpinv(pt)
        g = float(np.dot(res_like["grad_rs"], drs) + np.dot(res_like["grad_ps"], dps))
        errs["pinv"] = abs(g - pt["grad_pinv"]) / abs(pt["grad_pinv"])
    return errs
