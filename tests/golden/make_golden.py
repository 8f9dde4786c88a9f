#!/usr/bin/env python
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run in the build container (the reference is mounted at /root/reference; it
does not exist on the GPU box, so the fixtures are committed):

    python tests/golden/make_golden.py

What is taken from the reference (nothing here is restated by us):

* ``kat_3tax.json`` -- the closed-form 3-taxon JC log-likelihood of
  ``eigen/test_ll_3tax.py:22-320`` evaluated at the two points the script
  uses (``:323-329``), plus central finite-difference gradients of that same
  formula.  jax is absent, so ``jax`` / ``jax.numpy`` are bound to numpy for
  the duration of the import (the formula only calls ``exp`` and ``log``).
* ``phylo_gtr.json`` -- HKY / GTR log-likelihoods computed by the
  reference's own numpy pruner ``scripts/phylo.py`` (``GTR`` class
  ``:4-61``: normalised Q, ``numpy.linalg.eig``; ``traverse`` /
  ``compute_likelihood`` ``:240-296``: one rate category, every alignment
  column, tips one-hot or all-ones) on the fluA and HCV trees with their
  branch lengths times a clock rate.  The script is Python 2, so
  ``builtins.xrange`` is bound to ``range`` for the import; the tree and
  alignment objects are our DendroPy-compatible ones.  Per-site values are
  read from the reference's root partials exactly as ``compute_likelihood``
  forms them (``:285-290``).
* ``<dataset>_layout.npz`` -- the Stan data layout that ``phylostan run``
  builds: ``phylostan/utils.py`` functions ``setup_indexes``,
  ``setup_dates``, ``get_peeling_order``, ``get_preorder``, ``get_lowers``
  and ``get_dna_leaves_partials_compressed`` are imported from the reference
  and run on the example inputs.  DendroPy is absent, so the tree / alignment
  objects they walk are our own DendroPy-compatible ones
  (``phylostan_amd/treeio.py``); ``numpy.int`` (removed in numpy >= 1.24) is
  re-bound to ``int`` for the call.  ``tipdata`` (0/1 ``[S, L, 4]``) is
  stored losslessly as bit masks ``sum_k tipdata[..., k] << k``.
* ``DS1_topologies.npz`` -- config 1 over all 42 topologies of
  ``examples/DS1/DS1.trees``, as ``examples/SConstruct:159-188`` runs it:
  each topology's layout from ``utils.py`` and its per-site
  log-likelihoods from ``scripts/phylo.py`` (``ds1_topologies_fixture``).
"""
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from phylostan_amd import treeio  # noqa: E402


def _import_reference_utils():
    sys.path.insert(0, REF)
    import numpy
    if not hasattr(numpy, "int"):
        numpy.int = int
    from phylostan import utils  # noqa: E402  (pure python, needs numpy only)
    return utils


def kat_fixture():
    fake_jax = types.ModuleType("jax")
    fake_jax.numpy = np
    sys.modules["jax"] = fake_jax
    sys.modules["jax.numpy"] = np
    sys.path.insert(0, os.path.join(REF, "eigen"))
    import test_ll_3tax  # noqa: E402
    f = test_ll_3tax.loglik3tax
    mu = 1.0
    pi = np.ones(4) / 4
    tips = np.eye(4)[:3]
    points = []
    for times in ([1.0, 1.0, 1.0, 1.0], [0.1, 0.1, 0.2, 0.3]):
        t = np.array(times)
        ll = float(f(mu, pi, tips, t))
        h = 1e-6
        grad = []
        for k in range(4):
            tp, tm = t.copy(), t.copy()
            tp[k] += h
            tm[k] -= h
            grad.append((float(f(mu, pi, tips, tp)) - float(f(mu, pi, tips, tm))) / (2 * h))
        points.append({"branches_b14_b24_b45_b35": times, "loglik": ll, "grad_fd": grad})
    del sys.modules["jax"], sys.modules["jax.numpy"]
    return {
        "source": "eigen/test_ll_3tax.py:22-329 (reference closed form, evaluated with numpy)",
        "tree": "((1:b14,2:b24)4:b45,3:b35)5",
        "tips": "A, C, G (eye(4)[:3])",
        "Q": "JC unnormalised: off-diagonal 0.25, diagonal -0.75 (eigen/util.py:96-99); "
             "P(t) = 0.25 + 0.75 exp(-t) on the diagonal, so t_eigen = b_stan / 0.75",
        "points": points,
    }


class _Seq(str):
    def symbols_as_string(self):
        return str(self)


class _Alignment(dict):
    """What get_dna_leaves_partials_compressed touches of a DendroPy
    DnaCharacterMatrix: iteration in taxon-namespace order, ``[name][i]``,
    ``symbols_as_string()``, ``sequence_size``."""

    def __init__(self, rows):
        super().__init__(rows)
        self.sequence_size = len(next(iter(rows.values())))


def layout_fixture(utils, tree_path, aln_path, heterochronous, rooted):
    tree = treeio.read_tree(tree_path)
    tree.resolve_polytomies(update_bipartitions=True)
    utils.setup_indexes(tree)
    oldest = utils.setup_dates(tree, None, heterochronous)
    peel = utils.get_peeling_order(tree)
    if not rooted:  # phylostan.py:264-267
        last = peel[-1]
        if last[0] > last[1]:
            peel[-1] = [last[1], last[0], last[2]]
    pre = utils.get_preorder(tree)
    aln = treeio.read_alignment(aln_path)
    rows = {t.label: _Seq(aln[t.label]) for t in tree.taxon_namespace}
    tipdata, weights = utils.get_dna_leaves_partials_compressed(_Alignment(rows))
    tipdata = np.asarray(tipdata)
    bits = (tipdata * (1 << np.arange(4))).sum(-1).astype(np.uint8)
    out = dict(tipbits=bits, weights=np.asarray(weights, dtype=np.int64),
               peel=np.asarray(peel, dtype=np.int32), map=np.asarray(pre, dtype=np.int32),
               taxa=np.array([t.label for t in tree.taxon_namespace]),
               sites=np.int64(len(next(iter(aln.values())))))
    if heterochronous:
        out["lowers"] = np.asarray(utils.get_lowers(tree), dtype=np.float64)
        out["oldest"] = np.float64(oldest)
    # node heights implied by the input tree (used for fluA / HCV parameter
    # points: blens = rate * (h[parent] - h[node]), generate_script.py:660-679)
    S = len(tree.taxon_namespace)
    if any(n.edge_length is None for n in tree.postorder_node_iter() if n.parent_node is not None):
        return out  # topology-only tree (DS1)
    h = {}
    for node in tree.postorder_node_iter():
        h[node] = node.date if node.is_leaf() else max(h[c] + c.edge_length for c in node.child_node_iter())
    heights = np.zeros(S - 1)
    dates = np.zeros(S)
    for node in tree.postorder_node_iter():
        if node.is_leaf():
            dates[node.index - 1] = node.date
        else:
            heights[node.index - S - 1] = h[node]
    out["heights"] = heights
    out["tip_dates"] = dates
    return out


def _import_reference_phylo():
    import builtins
    if not hasattr(builtins, "xrange"):
        builtins.xrange = range
    sys.path.insert(0, os.path.join(REF, "scripts"))
    import phylo  # noqa: E402  (numpy + math only)
    return phylo


PHYLO_POINTS = [
    # dataset, model, exchangeabilities (AC AG AT CG CT GT), freqs (None = empirical), clock rate
    ("fluA", "HKY", [1.0, 5.58, 1.0, 1.0, 5.58, 1.0], None, 0.00499),
    ("fluA", "GTR", [1.2, 4.1, 0.7, 0.9, 5.3, 1.0], [0.31, 0.19, 0.23, 0.27], 0.004),
    ("HCV", "GTR", [0.125, 0.25, 0.125, 0.125, 0.25, 0.125], [0.25, 0.25, 0.25, 0.25], 7.9e-4),
    ("HCV", "HKY", [1.0, 3.0, 1.0, 1.0, 3.0, 1.0], [0.22, 0.28, 0.26, 0.24], 1.2e-3),
]


def phylo_gtr_fixture(utils, phylo, specs):
    """Log-likelihoods of the reference's scripts/phylo.py pruner."""
    from phylostan_amd import data, models
    out = {"source": "scripts/phylo.py:4-61 (GTR), :240-296 (traverse, compute_likelihood)",
           "convention": "one category; branch length = input-tree edge length * clock_rate; node ids "
                         "0-based as phylostan/utils.py setup_indexes minus one (tips in taxon-namespace "
                         "order, internal nodes in post-order); site_ll per compressed pattern of the "
                         "<dataset>_layout.npz fixture", "points": []}
    for name, model, rates, freqs, clock in PHYLO_POINTS:
        tpath, apath = specs[name][:2]
        tree = treeio.read_tree(tpath)
        tree.resolve_polytomies(update_bipartitions=True)
        aln = treeio.read_alignment(apath)
        rows = {t.label: _Seq(aln[t.label]) for t in tree.taxon_namespace}
        alignment = _Alignment(rows)  # iteration = taxon-namespace order
        for nd in tree.postorder_node_iter():
            if nd.parent_node is not None:
                nd.edge_length = nd.edge_length * clock
        layout = np.load(os.path.join(HERE, "%s_layout.npz" % name), allow_pickle=False)
        if freqs is None:
            freqs = models.empirical_frequencies(layout["tipbits"], layout["weights"]).tolist()
        gtr = phylo.GTR(list(rates), list(freqs))
        total = phylo.compute_likelihood(tree, alignment, gtr)
        # per-site values from the reference's own partials (compute_likelihood :283-290)
        S = len(alignment)
        partials = phylo.initialize_dna_partials(alignment)
        matrices = np.zeros((2 * S - 2, 4, 4))
        phylo.traverse(tree.seed_node, matrices, partials, gtr)
        root = partials[2 * S - 2]
        site = np.array([np.log(sum(root[i][j] * gtr.get_pi(j) for j in range(4)))
                         for i in range(alignment.sequence_size)])
        # map every site to its compressed pattern (first-seen order, raw symbols)
        chars = np.array([[ord(ch) for ch in str(rows[t.label]).upper()] for t in tree.taxon_namespace],
                         dtype=np.uint8)
        _, _, first = data.compress_patterns(chars)
        pat_ll = site[first]
        blens = np.zeros(2 * S - 2)
        for nd in tree.postorder_node_iter():
            if nd.parent_node is not None:
                blens[nd.index] = nd.edge_length
        out["points"].append({"dataset": name, "model": model, "rates": list(rates), "freqs": list(freqs),
                              "clock_rate": clock, "loglik": float(total), "site_ll": pat_ll.tolist(),
                              "blens": blens.tolist()})
        print(name, model, "reference loglik %.10f" % total)
    return out


def _phylo_root_site_lik(phylo, tree, alignment, gtr):
    """Per-site likelihoods L_i = sum_j pi_j p_root[i][j] from the
    reference's own post-order traversal (compute_likelihood :283-290)."""
    S = len(alignment)
    phylo.setup_indexes(tree, alignment)
    gtr.update()
    partials = phylo.initialize_dna_partials(alignment)
    matrices = np.zeros((2 * S - 2, 4, 4))
    phylo.traverse(tree.seed_node, matrices, partials, gtr)
    root = partials[2 * S - 2]
    return np.array([sum(root[i][j] * gtr.get_pi(j) for j in range(4)) for i in range(alignment.sequence_size)])


# The configs' own variants: the C = 4 Weibull mixture (fluA HKY+W4 at the
# README point, HCV GTR+W4 at SConstruct:218's) and DS1's unrooted JC69.
MIXTURE_POINTS = [
    # dataset, model, exchangeabilities, freqs (None = empirical), clock rate, Weibull shape
    ("fluA", "HKY", [1.0, 5.58, 1.0, 1.0, 5.58, 1.0], None, 0.00499, 0.488),
    ("HCV", "GTR", [0.125, 0.25, 0.125, 0.125, 0.25, 0.125], [0.25] * 4, 7.9e-4, 0.5),
]


def mixture_fixture(phylo, specs):
    """C = 4 Weibull mixtures and the unrooted merged-root-branch variant
    through the reference's scripts/phylo.py pruner.

    * Mixture (generate_script.py:998-1011): the reference pruner runs once
      per category with every edge scaled by r_c (P(b r_c), :876-880), and the
      per-site category likelihoods are combined as log sum_c ps_c L_c,i --
      the one line of :1006-1010 restated here; r_c, ps_c are the median
      Weibull categories of :267-278 (phylostan_amd.models.weibull_site_rates,
      itself checked against the literal restatement in tests/test_oracle.py).
    * DS1 (generate_script.py:1013-1023): the emitted code applies the root's
      first child's matrix only (the root branch merged into it) and uses
      node 2S-3's partials directly.  Under a reversible model the pulley
      principle makes that the likelihood of the rooted tree whose edge to
      node 2S-3 has length 0, so phylo.GTR([1]*6, [.25]*4) -- normalised JC69
      -- evaluates it on the resolved DS1 tree with that edge zeroed and
      blens ~ Exp(10) (seed 0, generate_script.py:1404) elsewhere.
    """
    from phylostan_amd import data, models
    out = {"source": "scripts/phylo.py:4-61 (GTR), :240-296 (traverse); mixture log sum_c ps_c L_c "
                     "(generate_script.py:1006-1010); unrooted = rooted with a zero root-edge to node 2S-3 "
                     "(generate_script.py:1019, pulley principle)", "points": []}

    def pattern_values(rows, taxa, site):
        chars = np.array([[ord(ch) for ch in str(rows[t]).upper()] for t in taxa], dtype=np.uint8)
        _, _, first = data.compress_patterns(chars)
        return site[first]

    for name, model, rates, freqs, clock, shape in MIXTURE_POINTS:
        tpath, apath = specs[name][:2]
        layout = np.load(os.path.join(HERE, "%s_layout.npz" % name), allow_pickle=False)
        if freqs is None:
            freqs = models.empirical_frequencies(layout["tipbits"], layout["weights"]).tolist()
        rs, ps = models.weibull_site_rates(shape, 4)
        aln = treeio.read_alignment(apath)
        lik = []
        for c in range(4):
            tree = treeio.read_tree(tpath)
            tree.resolve_polytomies(update_bipartitions=True)
            rows = {t.label: _Seq(aln[t.label]) for t in tree.taxon_namespace}
            alignment = _Alignment(rows)
            for nd in tree.postorder_node_iter():
                if nd.parent_node is not None:
                    nd.edge_length = nd.edge_length * clock * rs[c]
            lik.append(_phylo_root_site_lik(phylo, tree, alignment, phylo.GTR(list(rates), list(freqs))))
        site = np.log(sum(ps[c] * lik[c] for c in range(4)))
        taxa = [t.label for t in tree.taxon_namespace]
        S = len(taxa)
        blens = np.zeros(2 * S - 2)
        tree = treeio.read_tree(tpath)
        tree.resolve_polytomies(update_bipartitions=True)
        phylo.setup_indexes(tree, _Alignment({t.label: _Seq(aln[t.label]) for t in tree.taxon_namespace}))
        for nd in tree.postorder_node_iter():
            if nd.parent_node is not None:
                blens[nd.index] = nd.edge_length * clock
        out["points"].append({"dataset": name, "model": model, "rooted": True, "C": 4, "rates": list(rates),
                              "freqs": list(freqs), "rs": list(rs), "ps": list(ps), "clock_rate": clock,
                              "wshape": shape, "loglik": float(np.sum(site)),
                              "site_ll": pattern_values(rows, taxa, site).tolist(), "blens": blens.tolist()})
        print(name, model, "+W4 reference mixture loglik %.10f" % np.sum(site))
    # DS1 JC69 unrooted
    tpath, apath = specs["DS1"][:2]
    tree = treeio.read_tree(tpath)
    tree.resolve_polytomies(update_bipartitions=True)
    aln = treeio.read_alignment(apath)
    rows = {t.label: _Seq(aln[t.label]) for t in tree.taxon_namespace}
    alignment = _Alignment(rows)
    S = len(alignment)
    phylo.setup_indexes(tree, alignment)
    layout = np.load(os.path.join(HERE, "DS1_layout.npz"), allow_pickle=False)
    peel0 = layout["peel"] - 1
    assert peel0[-1][1] == 2 * S - 3
    blens = np.random.default_rng(0).exponential(1.0 / 10.0, size=2 * S - 3)  # tests/cases.py ds1_case(0)
    for nd in tree.postorder_node_iter():
        if nd.parent_node is not None:
            nd.edge_length = 0.0 if nd.index == 2 * S - 3 else float(blens[nd.index])
    # the merged branch: phylo's root children are peel0[-1][:2]
    root_children = sorted(c.index for c in tree.seed_node.child_node_iter())
    assert root_children == sorted(peel0[-1][:2].tolist()), (root_children, peel0[-1])
    site = np.log(_phylo_root_site_lik(phylo, tree, alignment, phylo.GTR([1.0] * 6, [0.25] * 4)))
    taxa = [t.label for t in tree.taxon_namespace]
    out["points"].append({"dataset": "DS1", "model": "JC69", "rooted": False, "C": 1, "rates": [1.0] * 6,
                          "freqs": [0.25] * 4, "rs": [1.0], "ps": [1.0], "loglik": float(np.sum(site)),
                          "site_ll": pattern_values(rows, taxa, site).tolist(), "blens": blens.tolist()})
    print("DS1 JC69 unrooted reference loglik %.10f" % np.sum(site))
    return out


def _pattern_alignment(layout, taxa):
    """The dataset's compressed patterns as an alignment object in the
    reference pruner's input form (one column per pattern; tip masks back to
    symbols: A C G T, '-' for the all-ones mask; the fixtures hold only
    one-hot and all-ones masks), plus the pattern weights."""
    sym = {1: "A", 2: "C", 4: "G", 8: "T", 15: "-"}
    tb = layout["tipbits"]
    assert set(np.unique(tb).tolist()) <= set(sym), "unexpected tip mask in the fixture"
    rows = {t: _Seq("".join(sym[int(v)] for v in tb[k])) for k, t in enumerate(taxa)}
    return _Alignment(rows), np.asarray(layout["weights"], dtype=np.float64)


def _ref_mixture_loglik(phylo, tree, alignment, weights, blens, rates, freqs, rs, ps, merged=None):
    """sum_i w_i log sum_c ps_c L_c,i with every L_c,i from the reference's
    scripts/phylo.py pruner (:240-296) on edges blens[node index] * r_c (the
    mixture line generate_script.py:1006-1010 restated); `merged`: the node
    whose edge is 0 (DS1's merged root branch, generate_script.py:1019)."""
    lik = 0.0
    for c in range(len(rs)):
        for nd in tree.postorder_node_iter():
            if nd.parent_node is not None:
                nd.edge_length = 0.0 if nd.index == merged else float(blens[nd.index]) * float(rs[c])
        lik = lik + float(ps[c]) * _phylo_root_site_lik(phylo, tree, alignment, phylo.GTR(list(rates), list(freqs)))
    return float(np.dot(weights, np.log(lik)))


GRAD_BRANCHES = 10  # branch-length derivatives per config point (spread over tip and internal branches)


def grad_fixture(phylo, specs):
    """Central differences of the reference's own likelihood (scripts/phylo.py
    pruner, mixture per generate_script.py:1006-1010) at the three configs'
    points: d/dblens for GRAD_BRANCHES branches, d/dkappa (fluA HKY) or the
    six GTR exchangeabilities (HCV), the four frequencies (as free
    variables: phylo.GTR uses them as given, so does the emitted Stan model,
    generate_script.py:855-868), and the Weibull shape through rs
    (:267-278).  Each derivative is Richardson-extrapolated from steps h and
    h/2 (truncation O(h^4)); the tests compare at rel 1e-6."""
    from phylostan_amd import models
    out = {"source": "central differences (Richardson, steps h and h/2) of scripts/phylo.py:240-296 "
                     "(per category) combined as generate_script.py:1006-1010", "points": []}

    def deriv(f, x0, h):
        d1 = (f(x0 + h) - f(x0 - h)) / (2 * h)
        d2 = (f(x0 + h / 2) - f(x0 - h / 2)) / h
        return (4.0 * d2 - d1) / 3.0

    with open(os.path.join(HERE, "phylo_mixture.json")) as fp:
        mix = {p["dataset"]: p for p in json.load(fp)["points"]}
    for name in ("fluA", "HCV", "DS1"):
        pt = mix[name]
        tpath, apath = specs[name][:2]
        layout = np.load(os.path.join(HERE, "%s_layout.npz" % name), allow_pickle=False)
        tree = treeio.read_tree(tpath)
        tree.resolve_polytomies(update_bipartitions=True)
        aln = treeio.read_alignment(apath)
        full = _Alignment({t.label: _Seq(aln[t.label]) for t in tree.taxon_namespace})
        phylo.setup_indexes(tree, full)
        taxa = [t.label for t in tree.taxon_namespace]
        alignment, w = _pattern_alignment(layout, taxa)
        S = len(taxa)
        merged = None if pt["rooted"] else 2 * S - 3
        blens = np.array(pt["blens"], dtype=np.float64)
        B = blens.size
        rates, freqs = list(pt["rates"]), list(pt["freqs"])
        rs, ps = list(pt["rs"]), list(pt["ps"])

        def F(bl=None, rt=None, fq=None, rsv=None):
            return _ref_mixture_loglik(phylo, tree, alignment, w, blens if bl is None else bl,
                                       rates if rt is None else rt, freqs if fq is None else fq,
                                       rs if rsv is None else rsv, ps, merged)

        ll0 = F()
        assert abs(ll0 - pt["loglik"]) <= 1e-9 * abs(pt["loglik"]), (ll0, pt["loglik"])
        rec = {"dataset": name, "model": pt["model"], "rooted": pt["rooted"], "C": pt["C"], "loglik": ll0}
        br = np.unique(np.linspace(0, B - 1, GRAD_BRANCHES).round().astype(int)).tolist()
        gb = []
        for b in br:
            h = 1e-3 * max(blens[b], 1e-4)

            def fb(x, b=b):
                bl = blens.copy()
                bl[b] = x
                return F(bl=bl)
            gb.append(deriv(fb, blens[b], h))
        rec["branches"] = br
        rec["grad_blens"] = gb
        if pt["model"] == "HKY":
            kappa = rates[1]
            rec["kappa"] = kappa
            rec["grad_kappa"] = deriv(lambda k: F(rt=[1.0, k, 1.0, 1.0, k, 1.0]), kappa, 1e-3 * kappa)
        if pt["model"] == "GTR":
            gr = []
            for k in range(6):
                def fr(x, k=k):
                    rt = list(rates)
                    rt[k] = x
                    return F(rt=rt)
                gr.append(deriv(fr, rates[k], 1e-3 * rates[k]))
            rec["grad_rates"] = gr
        if pt["model"] != "JC69":
            gf = []
            for k in range(4):
                def ff(x, k=k):
                    fq = list(freqs)
                    fq[k] = x
                    return F(fq=fq)
                gf.append(deriv(ff, freqs[k], 1e-4 * freqs[k]))
            rec["grad_freqs"] = gf
        if pt["C"] > 1:
            shape = pt["wshape"]
            rec["wshape"] = shape
            rec["grad_wshape"] = deriv(lambda a: F(rsv=list(models.weibull_site_rates(a, pt["C"])[0])), shape,
                                       1e-3 * shape)
        out["points"].append(rec)
        print(name, "reference FD gradients:", {k: v for k, v in rec.items() if k.startswith("grad")})
    return out


# Zero-rate and free-weight categories (site-rate variants other than the
# configs' plain Weibull): -I with Weibull (generate_script.py:250-266: rs[1] = 0,
# ps[1] = pinv), -I with one category (:1231-1240: C = 2, rs = (0, 1/(1-pinv))),
# and --heterogeneity discrete (:1221-1230: ps a simplex, rs = x / sum(ps .* x)).
ZERO_RATE_POINTS = [
    # dataset, model, kind, pinv / (ps, rate_unscaled), shape
    ("fluA", "HKY", "pinv_weibull", 0.2, 0.488),
    ("HCV", "GTR", "pinv_weibull", 0.3, 0.5),
    ("HCV", "GTR", "pinv_single", 0.25, None),
    ("fluA", "HKY", "discrete", ([0.1, 0.2, 0.3, 0.4], [0.05, 0.15, 0.3, 0.5]), None),
]


def _zero_rate_rates(kind, arg, shape):
    from phylostan_amd import models
    if kind == "pinv_weibull":
        return models.weibull_pinv_site_rates(shape, arg, 4)
    if kind == "pinv_single":
        return np.array([0.0, 1.0 / (1.0 - arg)]), np.array([arg, 1.0 - arg])
    ps, x = np.array(arg[0]), np.array(arg[1])
    return x / np.sum(ps * x), ps


def zero_rate_fixture(phylo, specs):
    """Log-likelihoods (total and per pattern) and central differences of the
    reference's scripts/phylo.py pruner (per category, edges b r_c -- a zero
    rate gives zero-length edges, P = I) combined as the mixture line
    generate_script.py:1006-1010, for the site-rate variants above: d/dpinv
    through rs and ps (the +I forms), d/drs_c and d/dps_c as free variables
    (every variant; at r_0 = 0 the central difference straddles zero), and
    four branch lengths.  Same points' data as the mixture fixture (fluA at
    the README point, HCV at SConstruct:218's)."""
    from phylostan_amd import models
    out = {"source": "scripts/phylo.py:240-296 per category, mixture generate_script.py:1006-1010; site rates "
                     "generate_script.py:250-266 (+I Weibull), :1231-1240 (+I, C = 1), :1221-1230 (discrete)",
           "points": []}

    def deriv(f, x0, h):
        d1 = (f(x0 + h) - f(x0 - h)) / (2 * h)
        d2 = (f(x0 + h / 2) - f(x0 - h / 2)) / h
        return (4.0 * d2 - d1) / 3.0

    with open(os.path.join(HERE, "phylo_mixture.json")) as fp:
        mix = {p["dataset"]: p for p in json.load(fp)["points"]}
    for name, model, kind, arg, shape in ZERO_RATE_POINTS:
        pt = mix[name]
        tpath, apath = specs[name][:2]
        layout = np.load(os.path.join(HERE, "%s_layout.npz" % name), allow_pickle=False)
        tree = treeio.read_tree(tpath)
        tree.resolve_polytomies(update_bipartitions=True)
        aln = treeio.read_alignment(apath)
        phylo.setup_indexes(tree, _Alignment({t.label: _Seq(aln[t.label]) for t in tree.taxon_namespace}))
        taxa = [t.label for t in tree.taxon_namespace]
        alignment, w = _pattern_alignment(layout, taxa)
        blens = np.array(pt["blens"], dtype=np.float64)
        rates, freqs = list(pt["rates"]), list(pt["freqs"])
        rs, ps = _zero_rate_rates(kind, arg, shape)

        def site(bl, rsv, psv):
            lik = 0.0
            for c in range(len(rsv)):
                for nd in tree.postorder_node_iter():
                    if nd.parent_node is not None:
                        nd.edge_length = float(bl[nd.index]) * float(rsv[c])
                lik = lik + float(psv[c]) * _phylo_root_site_lik(phylo, tree, alignment,
                                                                 phylo.GTR(list(rates), list(freqs)))
            return np.log(lik)

        def F(bl=blens, rsv=rs, psv=ps):
            return float(np.dot(w, site(bl, rsv, psv)))

        sl = site(blens, rs, ps)
        rec = {"dataset": name, "model": model, "kind": kind, "rooted": True, "C": len(rs), "rates": rates,
               "freqs": freqs, "rs": list(rs), "ps": list(ps), "blens": blens.tolist(),
               "loglik": float(np.dot(w, sl)), "site_ll": sl.tolist()}
        if kind != "discrete":
            rec["pinv"] = arg
            rec["grad_pinv"] = deriv(lambda x: F(rsv=_zero_rate_rates(kind, x, shape)[0],
                                                 psv=_zero_rate_rates(kind, x, shape)[1]), arg, 1e-4)
        if shape is not None:
            rec["wshape"] = shape
        grs, gps = [], []
        for c in range(len(rs)):
            def fr(x, c=c):
                r = np.array(rs, dtype=np.float64)
                r[c] = x
                return F(rsv=r)

            def fp_(x, c=c):
                q = np.array(ps, dtype=np.float64)
                q[c] = x
                return F(psv=q)
            if rs[c] == 0.0:  # phylo.GTR.p_t takes |P| (scripts/phylo.py:22): the reference has a kink
                # at t = 0, so the zero rate's derivative is one-sided (rates >= 0), forward Richardson
                h = 1e-6
                d1 = (fr(h) - fr(0.0)) / h
                d2 = (fr(h / 2) - fr(0.0)) / (h / 2)
                grs.append(2.0 * d2 - d1)
            else:
                grs.append(deriv(fr, rs[c], 1e-4 * rs[c]))
            gps.append(deriv(fp_, ps[c], 1e-4 * ps[c]))
        rec["grad_rs"], rec["grad_ps"] = grs, gps
        br = np.unique(np.linspace(0, blens.size - 1, 4).round().astype(int)).tolist()
        gb = []
        for b in br:
            def fb(x, b=b):
                bl = blens.copy()
                bl[b] = x
                return F(bl=bl)
            gb.append(deriv(fb, blens[b], 1e-3 * max(blens[b], 1e-4)))
        rec["branches"], rec["grad_blens"] = br, gb
        out["points"].append(rec)
        print(name, model, kind, "loglik %.10f" % rec["loglik"], {k: v for k, v in rec.items()
                                                                  if k.startswith("grad")})
    return out


DS1_LL_TOPOLOGIES = tuple(range(42))  # every topology gets reference per-site log-likelihoods


def ds1_topologies_fixture(utils, phylo):
    """Config 1 as the reference's pipeline runs it (examples/SConstruct:159-188):
    DS1.trees split into its 42 topologies, `phylostan run -m JC69` on each.
    For every line, the Stan data layout from the reference's own
    phylostan/utils.py (layout_fixture: peel with the unrooted swap of
    phylostan.py:264-267, map), the taxon-namespace order as a permutation of
    topology 0's (the compressed patterns do not depend on the row order:
    tipbits_k = tipbits_0[perm_k], checked here), and for every topology
    the per-pattern log-likelihoods of the reference's scripts/phylo.py pruner
    under the unrooted convention (the edge to node 2S-3 zeroed:
    generate_script.py:1019 and the pulley principle; normalised JC69) with
    blens ~ Exp(10), seed 1000 + k."""
    import tempfile
    from phylostan_amd import data
    tpath = os.path.join(REF, "examples", "DS1", "DS1.trees")
    apath = os.path.join(REF, "examples", "DS1", "DS1.nex")
    lines = [ln.rstrip("\n").rstrip("\r") for ln in open(tpath) if ln.strip()]
    aln = treeio.read_alignment(apath)
    out = {"peel": [], "map": [], "perm": [], "ll_topologies": list(DS1_LL_TOPOLOGIES), "blens": [], "site_ll": [],
           "loglik": []}
    taxa0 = tip0 = None
    with tempfile.TemporaryDirectory() as td:
        for k, line in enumerate(lines):
            tf = os.path.join(td, "tree%d.tree" % k)
            with open(tf, "w") as fp:
                fp.write(line)
            fx = layout_fixture(utils, tf, apath, False, False)
            taxa = [str(t) for t in fx["taxa"]]
            if k == 0:
                taxa0, tip0 = taxa, fx["tipbits"]
                out["taxa0"] = taxa0
                out["tipbits0"] = tip0
                out["weights"] = fx["weights"]
            perm = np.array([taxa0.index(t) for t in taxa], dtype=np.int32)
            assert np.array_equal(fx["tipbits"], tip0[perm]), "patterns depend on the row order"
            out["peel"].append(fx["peel"])
            out["map"].append(fx["map"])
            out["perm"].append(perm)
            if k in DS1_LL_TOPOLOGIES:
                tree = treeio.read_tree(tf)
                tree.resolve_polytomies(update_bipartitions=True)
                rows = {t.label: _Seq(aln[t.label]) for t in tree.taxon_namespace}
                alignment = _Alignment(rows)
                S = len(alignment)
                phylo.setup_indexes(tree, alignment)
                peel0 = fx["peel"] - 1
                assert peel0[-1][1] == 2 * S - 3
                blens = np.random.default_rng(1000 + k).exponential(1.0 / 10.0, size=2 * S - 3)
                for nd in tree.postorder_node_iter():
                    if nd.parent_node is not None:
                        nd.edge_length = 0.0 if nd.index == 2 * S - 3 else float(blens[nd.index])
                site = np.log(_phylo_root_site_lik(phylo, tree, alignment, phylo.GTR([1.0] * 6, [0.25] * 4)))
                chars = np.array([[ord(ch) for ch in str(rows[t]).upper()] for t in taxa], dtype=np.uint8)
                _, _, first = data.compress_patterns(chars)
                out["blens"].append(blens)
                out["site_ll"].append(site[first])
                out["loglik"].append(float(np.sum(site)))
                print("DS1 topology %d JC69 unrooted reference loglik %.10f" % (k, np.sum(site)))
    return {"peel": np.stack(out["peel"]), "map": np.stack(out["map"]), "perm": np.stack(out["perm"]),
            "taxa0": np.array(out["taxa0"]), "tipbits0": out["tipbits0"], "weights": out["weights"],
            "ll_topologies": np.array(out["ll_topologies"], dtype=np.int32), "blens": np.stack(out["blens"]),
            "site_ll": np.stack(out["site_ll"]), "loglik": np.array(out["loglik"])}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "zero_rate":  # only the site-rate variants' fixture
        ex = os.path.join(REF, "examples")
        specs = {"fluA": (os.path.join(ex, "fluA", "fluA.tree"), os.path.join(ex, "fluA", "fluA.fa")),
                 "HCV": (os.path.join(ex, "HCV", "HCV.tree"), os.path.join(ex, "HCV", "HCV.nexus"))}
        with open(os.path.join(HERE, "phylo_zero_rate.json"), "w") as fp:
            json.dump(zero_rate_fixture(_import_reference_phylo(), specs), fp)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "grad":  # only the reference FD gradients
        ex = os.path.join(REF, "examples")
        specs = {"fluA": (os.path.join(ex, "fluA", "fluA.tree"), os.path.join(ex, "fluA", "fluA.fa")),
                 "HCV": (os.path.join(ex, "HCV", "HCV.tree"), os.path.join(ex, "HCV", "HCV.nexus")),
                 "DS1": (os.path.join(ex, "DS1", "DS1.trees"), os.path.join(ex, "DS1", "DS1.nex"))}
        with open(os.path.join(HERE, "phylo_grad.json"), "w") as fp:
            json.dump(grad_fixture(_import_reference_phylo(), specs), fp, indent=1)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "ds1_topologies":  # only the 42 DS1 topologies
        np.savez_compressed(os.path.join(HERE, "DS1_topologies.npz"),
                            **ds1_topologies_fixture(_import_reference_utils(), _import_reference_phylo()))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "mixture":  # only the mixture / unrooted fixture
        ex = os.path.join(REF, "examples")
        specs = {"fluA": (os.path.join(ex, "fluA", "fluA.tree"), os.path.join(ex, "fluA", "fluA.fa")),
                 "HCV": (os.path.join(ex, "HCV", "HCV.tree"), os.path.join(ex, "HCV", "HCV.nexus")),
                 "DS1": (os.path.join(ex, "DS1", "DS1.trees"), os.path.join(ex, "DS1", "DS1.nex"))}
        with open(os.path.join(HERE, "phylo_mixture.json"), "w") as fp:
            json.dump(mixture_fixture(_import_reference_phylo(), specs), fp)
        return
    with open(os.path.join(HERE, "kat_3tax.json"), "w") as fp:
        json.dump(kat_fixture(), fp, indent=1)
    utils = _import_reference_utils()
    ex = os.path.join(REF, "examples")
    specs = {
        "fluA": (os.path.join(ex, "fluA", "fluA.tree"), os.path.join(ex, "fluA", "fluA.fa"), True, True),
        "HCV": (os.path.join(ex, "HCV", "HCV.tree"), os.path.join(ex, "HCV", "HCV.nexus"), False, True),
        "DS1": (os.path.join(ex, "DS1", "DS1.trees"), os.path.join(ex, "DS1", "DS1.nex"), False, False),
    }
    for name, (tpath, apath, het, rooted) in specs.items():
        fx = layout_fixture(utils, tpath, apath, het, rooted)
        np.savez_compressed(os.path.join(HERE, "%s_layout.npz" % name), **fx)
        print(name, "S=%d P=%d sites=%d" % (fx["tipbits"].shape[0], fx["tipbits"].shape[1], fx["sites"]))
    phylo = _import_reference_phylo()
    with open(os.path.join(HERE, "phylo_gtr.json"), "w") as fp:
        json.dump(phylo_gtr_fixture(utils, phylo, specs), fp)
    with open(os.path.join(HERE, "phylo_mixture.json"), "w") as fp:
        json.dump(mixture_fixture(phylo, specs), fp)
    np.savez_compressed(os.path.join(HERE, "DS1_topologies.npz"), **ds1_topologies_fixture(utils, phylo))


if __name__ == "__main__":
    main()
