"""The phylostan posterior on the host, with its exact gradient.

This is the Stan program ``phylostan/generate_script.py:get_model``
(``:1168-1484``) emits, minus the tree likelihood, which is the GPU engine
(``TreeLikelihood``): the parameter blocks, their constraining transforms,
the transformed parameters (site rates, node heights, branch lengths), the
priors and the log-Jacobian of the height reparametrisation.  Its gradient is
assembled by hand (reverse mode) around the engine's outputs:

  dlogL/dblens   -> rate (strict) or per-branch substrates (relaxed clocks),
                    node heights -> props, root height
  dlogL/drs, /dps-> Weibull shape (+ pinv), or the discrete-rate simplices
  dlogL/dP[c][b] -> kappa / GTR exchangeabilities and frequencies through the
                    eigendecomposition (``models.q_param_gradients``)

Parameter order, names and supports are Stan's (``:1212-1418``); the
unconstrained vector is laid out in that order, so a draw maps onto the
columns a Stan sample CSV would hold.

Supported ``build`` options (``phylostan/phylostan.py:69-95``): models JC69 /
HKY / GTR; ``-C`` Weibull categories (+ ``--invariant``) or ``--heterogeneity
discrete``; no clock (unrooted, ``blens ~ exponential(10)``), ``--clock
strict`` with ``--estimate_rate`` or a fixed ``--rate``, or a relaxed clock
(``ucln``, ``uced``, ``ace``, ``acln``, ``acg``, ``aoup``, ``gmrf``,
``hsmrf``; ``clocks.py``); ``--coalescent`` constant / skyride / skygrid;
``--speciation bd`` (``yule`` adds nothing, as emitted); ``--heterochronous``.
Phylogeography (``--geo``) is refused loudly.
"""
import math
import os

import numpy as np

from . import clocks
from . import hostlib
from . import models
from . import priors
from . import transforms
from .transforms import Identity, Lower, Simplex, Unit


class ModelSpec:
    """The ``build``/``run`` options that shape the model."""

    def __init__(self, model="GTR", categories=1, invariant=False, heterogeneity="weibull",
                 clock=None, estimate_rate=False, coalescent=None, heterochronous=False,
                 rate=None, lower_root=0.0, grid=None, cutoff=None, speciation=None):
        if model not in models.MODEL_IDS:
            raise ValueError("model must be JC69, HKY or GTR")
        if clock not in (None, "strict") + clocks.RELAXED:
            raise ValueError("unknown clock %r" % clock)
        if clock in clocks.AUTOCORR and not estimate_rate:
            # heights_to_blens_autocorr reads substrates, which only exist
            # with --estimate_rate: the emitted model would not compile
            raise ValueError("clock %r needs --estimate_rate" % clock)
        if speciation not in (None, "bd", "yule"):
            raise ValueError("unknown speciation model %r" % speciation)
        if speciation is not None and clock is None:
            raise ValueError("a speciation prior needs a clock")
        if coalescent not in (None, "constant", "skyride", "skygrid"):
            raise ValueError("unknown coalescent %r" % coalescent)
        if clock is None and coalescent is not None:
            raise ValueError("a coalescent prior needs a clock")
        if coalescent == "skygrid" and (grid is None or cutoff is None):
            raise ValueError("skygrid needs --grid and --cutoff")
        if invariant and categories > 1 and heterogeneity != "weibull":
            raise ValueError("Cannot use proportion of invariant and discrete rate heterogeneity yet.")
        self.model = model
        self.categories = int(categories)
        self.invariant = bool(invariant)
        self.heterogeneity = heterogeneity
        self.clock = clock
        self.estimate_rate = bool(estimate_rate)
        self.coalescent = coalescent
        self.heterochronous = bool(heterochronous)
        self.rate = None if rate is None else float(rate)
        self.lower_root = float(lower_root)
        self.grid = grid
        self.cutoff = cutoff
        self.speciation = speciation

    @property
    def relaxed(self):
        """A relaxed clock with per-branch substrates (needs --estimate_rate;
        without it ucln/uced fall back to the strict blens, as emitted)."""
        return self.clock in clocks.RELAXED and self.estimate_rate

    @property
    def C(self):
        """Rate categories the likelihood sees (data ``C``, phylostan.py:269-272)."""
        if self.categories > 1:
            return self.categories + (1 if self.invariant else 0)
        return 2 if self.invariant else 1

    @classmethod
    def from_args(cls, a):
        return cls(model=a.model, categories=a.categories, invariant=a.invariant,
                   heterogeneity=getattr(a, "heterogeneity", "weibull"), clock=a.clock,
                   estimate_rate=a.estimate_rate, coalescent=a.coalescent,
                   heterochronous=a.heterochronous, rate=getattr(a, "rate", None),
                   lower_root=getattr(a, "lower_root", 0.0) or 0.0, grid=getattr(a, "grid", None),
                   cutoff=getattr(a, "cutoff", None), speciation=getattr(a, "speciation", None))


class _Param:
    def __init__(self, name, transform):
        self.name = name
        self.tr = transform
        self.sl = None

    def names(self):
        if not self.tr.shape:
            return [self.name]
        return ["%s.%d" % (self.name, k + 1) for k in range(self.tr.shape[0])]


class TreeData:
    """The arrays of the Stan data dict the posterior needs (1-based ``map``
    like ``utils.get_preorder``; ``lowers`` indexed by 0-based node id)."""

    def __init__(self, S, peel0, map1, lowers=None, oldest=None):
        self.S = int(S)
        self.peel0 = np.asarray(peel0, np.int64)
        self.map1 = np.asarray(map1, np.int64)
        self.lowers = None if lowers is None else np.asarray(lowers, np.float64)
        self.oldest = oldest

    @classmethod
    def from_phylodata(cls, d):
        return cls(d.S, d.peel0, d.map, d.lowers, d.oldest)


class Posterior:
    """log p(theta | data) up to Stan's ``~`` constants, batched over draws.

    ``likelihood`` is any object with ``evaluate_batch(blens [n,B],
    model_vecs [n,10+2C]) -> [EvalResult]`` -- the GPU ``TreeLikelihood`` in
    the product.  ``compact_rows=True`` switches that likelihood to compact
    output rows (``set_output(compact=True)``: no dL/dP block, which the
    posterior never reads) -- a change to the caller's object, so it is
    opt-in; the CLI and the samplers' drivers ask for it.
    """

    def __init__(self, spec, tree, likelihood, compact_rows=False):
        self.spec = spec
        self.tree = tree
        self.lik = likelihood
        if compact_rows and hasattr(likelihood, "set_output"):
            likelihood.set_output(compact=True)
        S = tree.S
        self.S = S
        self.C = spec.C
        self.clock = spec.clock is not None
        self.B = 2 * S - 2 if self.clock else 2 * S - 3
        self._setup_tree()
        self.params = self._declare()
        off = 0
        for p in self.params:
            p.sl = slice(off, off + p.tr.size)
            off += p.tr.size
        self.dim = off
        self.const = self._dropped_constants()
        i = np.arange(1, self.C + 1, dtype=np.float64)
        self._wx = -np.log(1.0 - (2.0 * (i - 1) + 1.0) / (2.0 * self.C))  # Weibull quantile bases
        self._fast = self._native_strict()

    def _native_strict(self):
        """The native two-phase log density (hostlib.StrictPosterior) for the
        strict-clock family it covers -- phylostan's default build (Weibull
        or no site rates, any substitution model, estimated or fixed rate,
        constant coalescent or none) -- else None (the numpy path below,
        which stays the specification).  PHYLO_HOST_FAST=0 turns it off."""
        sp = self.spec
        lib = hostlib.load()
        if (getattr(self, "_nat", None) is None or lib is None or not hasattr(lib, "phh_strict_create")
                or os.environ.get("PHYLO_HOST_FAST", "1") == "0"):
            return None
        if (sp.clock != "strict" or sp.coalescent not in (None, "constant") or sp.speciation not in (None, "yule")
                or sp.invariant or (sp.categories > 1 and sp.heterogeneity != "weibull") or self.C > 64):
            return None
        off = {p.name: p.sl.start for p in self.params}
        names = ["wshape", "props", "rate", "height", "theta", "kappa", "rates", "freqs"]
        offsets = [off.get(k, -1) for k in names]
        fixed = sp.rate if sp.rate is not None else 1.0
        return hostlib.StrictPosterior(self._nat, self.S, self.B, self.C, models.MODEL_IDS[sp.model],
                                       sp.categories > 1, sp.estimate_rate, fixed, sp.coalescent == "constant",
                                       sp.heterochronous, self.lower_root, self.dim, offsets, self.lowers)

    # ------------------------------------------------------------------ layout
    def _declare(self):
        sp = self.spec
        P = []
        if sp.categories > 1 and sp.heterogeneity == "weibull":
            P.append(_Param("wshape", Lower(0.1)))
            if sp.invariant:
                P.append(_Param("pinv", Unit()))
        elif sp.categories > 1 and not sp.invariant:
            P.append(_Param("ps", Simplex(sp.categories)))
            P.append(_Param("rate_unscaled", Simplex(sp.categories)))
        elif sp.invariant and sp.categories == 1:
            P.append(_Param("pinv", Unit()))
        if self.clock:
            P.append(_Param("props", Unit(self.S - 2)))
            if sp.estimate_rate:
                if sp.clock == "strict":
                    P.append(_Param("rate", Lower(0.0)))
                elif sp.clock in clocks.MRF:
                    P.append(_Param("deltas", Identity(2 * self.S - 3)))
                    P.append(_Param("rate", Lower(0.0)))
                    P.append(_Param("zeta", Lower(0.0)))
                    if sp.clock == "hsmrf":
                        P.append(_Param("gammas", Lower(0.0, self.B - 1)))
                else:
                    P.append(_Param("substrates", Lower(0.0, self.B)))
                    if sp.clock in ("acln", "acg"):
                        P.append(_Param("nu", Lower(0.0)))
                    elif sp.clock == "aoup":
                        P.append(_Param("beta", Lower(0.0)))
                        P.append(_Param("sigma", Lower(0.0)))
                    elif sp.clock == "ucln":
                        P.append(_Param("ucln_mean", Lower(0.0)))
                        P.append(_Param("ucln_stdev", Lower(0.0)))
                    elif sp.clock == "uced":
                        P.append(_Param("uced_mean", Lower(0.0)))
            P.append(_Param("height", Lower(self.lower_root)))
            if sp.coalescent == "constant":
                P.append(_Param("theta", Lower(0.0)))
            elif sp.coalescent == "skyride":
                P.append(_Param("thetas", Identity(self.S - 1)))
                P.append(_Param("tau", Lower(0.0)))
            elif sp.coalescent == "skygrid":
                P.append(_Param("thetas", Identity(int(sp.grid) - 1)))
                P.append(_Param("tau", Lower(0.0)))
            if sp.speciation == "bd":
                P.append(_Param("netDiversificationRate", Lower(0.0)))
                P.append(_Param("relativeExtinctionRate", Unit()))
        else:
            P.append(_Param("blens", Lower(0.0, self.B)))
        if sp.model == "GTR":
            P.append(_Param("rates", Simplex(6)))
            P.append(_Param("freqs", Simplex(4)))
        elif sp.model == "HKY":
            P.append(_Param("kappa", Lower(0.0)))
            P.append(_Param("freqs", Simplex(4)))
        return P

    def param(self, name):
        for p in self.params:
            if p.name == name:
                return p
        return None

    def unconstrained_names(self):
        out = []
        for p in self.params:
            out += ["%s[%d]" % (p.name, k) for k in range(p.tr.size)] if p.tr.size > 1 or p.tr.shape \
                else [p.name]
        return out

    def _setup_tree(self):
        """Pre-order (map) bookkeeping for heights / blens (0-based ids)."""
        S = self.S
        t = self.tree
        if not self.clock:
            return
        m = t.map1 - 1  # [node, parent]; root row parent -1
        self.root = int(m[0, 0])
        self.lowers = np.zeros(2 * S - 1) if t.lowers is None else np.asarray(t.lowers, np.float64)
        if self.spec.heterochronous:
            oldest = t.oldest if t.oldest is not None else float(self.lowers[:S].max())
            self.lower_root = max(float(oldest), self.spec.lower_root)
        else:
            self.lower_root = self.spec.lower_root
        parent = np.full(2 * S - 1, -1, np.int64)
        depth = np.zeros(2 * S - 1, np.int64)
        prop_of = np.full(2 * S - 1, -1, np.int64)
        j = 0
        for node, par in m[1:]:
            parent[node] = par
            depth[node] = depth[par] + 1
            if node >= S:
                prop_of[node] = j
                j += 1
        if j != S - 2:
            raise ValueError("map does not list S-2 non-root internal nodes")
        self.parent = parent
        self.prop_of = prop_of
        internal = np.arange(S, 2 * S - 1)
        nonroot_int = internal[internal != self.root]
        # levels of non-root internal nodes, top-down (parents before children)
        self.levels = []
        for d in range(1, int(depth.max()) + 1):
            nodes = nonroot_int[depth[nonroot_int] == d]
            if len(nodes):
                self.levels.append((nodes, parent[nodes] - S, prop_of[nodes], self.lowers[nodes]))
        self.nonroot_int = nonroot_int
        bnodes = np.arange(self.B)  # every non-root node's branch
        if self.root != 2 * S - 2:
            raise ValueError("root must be node 2S-1 (1-based)")
        self.b_parent = parent[bnodes] - S
        self.b_internal = bnodes >= S
        self.b_hidx = np.where(self.b_internal, bnodes - S, 0)
        self.b_lower = self.lowers[bnodes]
        self.times_internal = np.zeros(2 * S - 1, bool)
        self.times_internal[S:] = True
        self.ctree = clocks.ClockTree(S, t.map1) if self.spec.relaxed else None
        # native routines for the same loops (hostlib), when built
        self._nat = None
        if hostlib.load() is not None and os.environ.get("PHYLO_HOST_NATIVE", "1") != "0":
            cat = (lambda k: np.concatenate([lv[k] for lv in self.levels])) if self.levels else \
                (lambda k: np.zeros(0))
            self._nat = hostlib.ClockTreeNative(
                S, cat(0) - S, cat(1), cat(2), cat(3), self.root - S, self.b_parent, self.b_hidx, self.b_internal,
                self.b_lower, parent[nonroot_int] - S, self.lowers[nonroot_int])

    def _dropped_constants(self):
        """Normalising constants Stan's ``~`` statements drop (propto) -- added
        back for ``log_prob(propto=False)``, which ADVI's ELBO uses."""
        sp = self.spec
        c = 0.0
        if sp.categories > 1 and sp.heterogeneity == "weibull":
            c += math.log(1.0)  # wshape ~ exponential(1)
        if self.clock:
            if sp.estimate_rate and sp.clock == "strict":
                c += math.log(1000.0)
            if sp.relaxed:
                c += clocks.dropped_constants(sp.clock, self.B, 2 * self.S - 3)
            if sp.coalescent in ("skyride", "skygrid"):
                a = b = 0.001
                c += -math.lgamma(a) + a * math.log(b)
        else:
            c += self.B * math.log(10.0)
        if sp.model in ("GTR", "HKY"):
            c += math.lgamma(4.0)  # dirichlet(1,1,1,1)
        if sp.model == "GTR":
            c += math.lgamma(6.0)
        if sp.model == "HKY":
            c += -math.log(1.25) - 0.5 * math.log(2.0 * math.pi)
        return c

    # --------------------------------------------------------------- forward
    def constrain(self, U):
        U = np.atleast_2d(np.asarray(U, np.float64))
        vals, states, logj = {}, {}, np.zeros(U.shape[0])
        for p in self.params:
            x, lj, st = p.tr.constrain(U[:, p.sl])
            vals[p.name] = x
            states[p.name] = st
            logj = logj + lj
        return vals, states, logj

    def _site_rates(self, vals, n):
        """rs, ps [n, C] and the pieces their gradients need."""
        sp = self.spec
        C = self.C
        if sp.categories > 1 and sp.heterogeneity == "weibull":
            w = vals["wshape"]
            if sp.invariant:
                pinv = vals["pinv"]
                rs = np.empty((n, C))
                ps = np.empty((n, C))
                for d in range(n):
                    rs[d], ps[d] = models.weibull_pinv_site_rates(w[d], pinv[d], C)
                return rs, ps
            # models.weibull_site_rates, all draws at once
            g = np.power(self._wx[None, :], 1.0 / w[:, None])
            return g / (g.sum(axis=1, keepdims=True) / C), np.full((n, C), 1.0 / C)
        if sp.categories > 1:
            ps = vals["ps"]
            ru = vals["rate_unscaled"]
            tot = (ps * ru).sum(axis=1, keepdims=True)
            return ru / tot, ps.copy()
        if sp.invariant:
            pinv = vals["pinv"]
            rs = np.stack([np.zeros(n), 1.0 / (1.0 - pinv)], axis=1)
            ps = np.stack([pinv, 1.0 - pinv], axis=1)
            return rs, ps
        return np.ones((n, 1)), np.ones((n, 1))

    def _lik_rows(self, blens, mv):
        """The likelihood's output rows [n, >= 1 + B + 2C + 14] (the engine's
        raw rows when it offers them, else assembled from EvalResult objects)."""
        if hasattr(self.lik, "evaluate_rows"):
            return self.lik.evaluate_rows(blens, mv)
        return np.stack([np.concatenate([[r.loglik], r.grad_blens, r.grad_rs, r.grad_ps, r.grad_freq_root,
                                         r.grad_rates, r.grad_freqs]) for r in self.lik.evaluate_batch(blens, mv)])

    def _heights(self, vals, n):
        if self._nat is not None:
            return self._nat.heights(vals["props"], vals["height"])
        S = self.S
        h = np.empty((n, S - 1))
        h[:, self.root - S] = vals["height"]
        props = vals["props"]
        for nodes, pidx, jidx, low in self.levels:
            h[:, nodes - S] = low + (h[:, pidx] - low) * props[:, jidx]
        return h

    def _span(self, h):
        """Branch durations [n, B]: heights[parent] - heights[node] (tips: - lowers)."""
        if self._nat is not None:
            return self._nat.span(h)
        base = np.where(self.b_internal, h[:, self.b_hidx], self.b_lower)
        return h[:, self.b_parent] - base

    def _substrates(self, vals):
        """Per-branch substrates of a relaxed clock [n, B] (MRF: transformed
        from deltas and rate, get_rates_from_deltas)."""
        if self.spec.clock in clocks.MRF:
            return clocks.rates_from_deltas(self.ctree, vals["deltas"], vals["rate"])
        return vals["substrates"]

    def _multiplier(self, vals, n):
        """blens = span * mult: (mult [n, B], substrates or None)."""
        if self.spec.relaxed:
            r = self._substrates(vals)
            return clocks.blens_multiplier(self.ctree, self.spec.clock, r), r
        return np.repeat(self._rate(vals, n)[:, None], self.B, axis=1), None

    def _rate(self, vals, n):
        if self.spec.estimate_rate:
            return vals["rate"]
        return np.full(n, self.spec.rate if self.spec.rate is not None else 1.0)

    def _q_params(self, vals, n):
        sp = self.spec
        if sp.model == "GTR":
            return vals["freqs"], vals["rates"]
        if sp.model == "HKY":
            k = vals["kappa"]
            R = np.ones((n, 6))
            R[:, 1] = k
            R[:, 4] = k
            return vals["freqs"], R
        return np.full((n, 4), 0.25), np.ones((n, 6))

    def transformed(self, U):
        """The constrained parameters and Stan's transformed parameters, in
        the order a Stan sample CSV lists them: [(name, [n, ...]), ...]."""
        U = np.atleast_2d(np.asarray(U, np.float64))
        n = U.shape[0]
        vals, _, _ = self.constrain(U)
        out = [(p.name, vals[p.name]) for p in self.params]
        sp = self.spec
        rs, ps = self._site_rates(vals, n)
        if sp.categories > 1 and sp.heterogeneity == "weibull":
            out += [("ps", ps), ("rs", rs)]
        elif sp.categories > 1:
            cons = vals["ps"] * vals["rate_unscaled"]
            out += [("rs", rs), ("constraint", cons / cons.sum(axis=1, keepdims=True))]
        elif sp.invariant:
            out += [("ps", ps), ("rs", rs)]
        if self.clock:
            out.append(("heights", self._heights(vals, n)))
            if sp.relaxed and sp.clock in clocks.MRF:
                out.append(("substrates", self._substrates(vals)))
        return out

    def blens(self, U):
        """Branch lengths [n, B] (model-block local ``blens``)."""
        U = np.atleast_2d(np.asarray(U, np.float64))
        n = U.shape[0]
        vals, _, _ = self.constrain(U)
        if not self.clock:
            return vals["blens"]
        return self._span(self._heights(vals, n)) * self._multiplier(vals, n)[0]

    # ------------------------------------------------------- value + gradient
    def in_support(self, U):
        """Rows of U whose constrained parameters are finite and strictly
        inside their declared bounds (a draw outside is a Stan domain
        error: rejected with lp = -inf before anything is evaluated)."""
        U = np.atleast_2d(np.asarray(U, np.float64))
        with np.errstate(all="ignore"):
            return self._support(U, *self.constrain(np.where(np.isfinite(U), U, 0.0)))[0]

    def _bounds(self):
        """Strict open bounds (lo, hi) of every constrained coordinate."""
        lo, hi = [], []
        for p in self.params:
            k = int(np.prod(p.tr.shape)) if p.tr.shape else 1
            if isinstance(p.tr, transforms.Lower):
                a, b = p.tr.lower, np.inf
            elif isinstance(p.tr, transforms.Unit):
                a, b = 0.0, 1.0
            elif isinstance(p.tr, transforms.Simplex):
                a, b = 0.0, np.inf
            else:
                a, b = -np.inf, np.inf
            lo += [a] * k
            hi += [b] * k
        return np.array(lo), np.array(hi)

    def _support(self, U, vals, states, logj):
        """in_support on already-constrained values (one vector test)."""
        n = U.shape[0]
        if not hasattr(self, "_lo"):
            self._lo, self._hi = self._bounds()
        X = np.concatenate([np.asarray(vals[p.name], np.float64).reshape(n, -1) for p in self.params], axis=1)
        ok = (np.isfinite(U).all(axis=1) & np.isfinite(logj)
              & (np.isfinite(X) & (X > self._lo) & (X < self._hi)).all(axis=1))
        return ok, vals, states, logj

    def log_prob_grad(self, U, propto=True, need_grad=True):
        """(lp [n], grad [n, dim]) at unconstrained draws U [n, dim]
        (Jacobian included, as Stan's ``log_prob<propto, jacobian=true>``).

        Out-of-support draws (``in_support``) are rejected up front: lp =
        -inf, zero gradient, and neither the transforms' numpy nor the GPU
        sees them.  Draws in support whose arithmetic still overflows are
        rejected the same way after evaluation."""
        return self.log_prob_grad_end(self.log_prob_grad_begin(U, propto, need_grad))

    def log_prob_grad_begin(self, U, propto=True, need_grad=True):
        """First half of ``log_prob_grad``: the host work up to the likelihood,
        whose evaluation is started (asynchronously when the engine offers
        ``submit_rows``); ``log_prob_grad_end`` finishes.  Lets a sampler
        overlap one group of chains' host work with another's GPU work."""
        if self._fast is not None:
            U = np.ascontiguousarray(np.atleast_2d(U), np.float64)
            cnt, bl, mv, sel = self._fast.pre(U)
            tok = {"fast": True, "U": U, "sel": sel, "propto": propto, "need_grad": need_grad}
            if cnt:
                if hasattr(self.lik, "submit_rows") and cnt <= min(getattr(self.lik, "max_draws", 64),
                                                                   getattr(self.lik, "_STAGE_DRAWS", 64)):
                    self.lik.submit_rows(bl, mv)
                    tok["async"] = True
                else:
                    tok["rows"] = self._lik_rows(bl, mv)
            return tok
        U = np.atleast_2d(np.asarray(U, np.float64))
        n = U.shape[0]
        with np.errstate(all="ignore"):
            ok, vals, states, logj = self._support(U, *self.constrain(np.where(np.isfinite(U), U, 0.0)))
        tok = {"n": n, "ok": ok, "need_grad": need_grad, "gen": None}
        if ok.any():
            pre = (vals, states, logj) if ok.all() else None  # the usual case: the constrained values are reused
            gen = self._lpg_gen(U[ok], propto, need_grad, pre)
            try:
                with np.errstate(over="ignore", under="ignore"):
                    req = next(gen)
            except StopIteration as e:
                tok["done"] = e.value
                return tok
            tok["gen"] = gen
            if hasattr(self.lik, "submit_rows") and req[0].shape[0] <= min(getattr(self.lik, "max_draws", 64),
                                                                            getattr(self.lik, "_STAGE_DRAWS", 64)):
                self.lik.submit_rows(*req)
                tok["async"] = True
            else:
                with np.errstate(over="ignore", under="ignore"):
                    tok["rows"] = self._lik_rows(*req)
        return tok

    def log_prob_grad_end(self, tok):
        if tok.get("fast"):
            rows = self.lik.wait_rows() if tok.get("async") else tok.get("rows")
            lp, G = self._fast.post(tok["U"], rows, tok["sel"], tok["need_grad"])
            if not tok["propto"]:
                lp = np.where(np.isfinite(lp), lp + self.const, lp)
            return lp, G
        n, ok, need_grad = tok["n"], tok["ok"], tok["need_grad"]
        lp = np.full(n, -np.inf)
        G = np.zeros((n, self.dim)) if need_grad else None
        res = tok.get("done")
        if tok["gen"] is not None:
            rows = self.lik.wait_rows() if tok.get("async") else tok["rows"]
            try:
                with np.errstate(over="ignore", under="ignore"):
                    tok["gen"].send(rows)
                raise RuntimeError("internal: log-density generator did not finish")
            except StopIteration as e:
                res = e.value
        if res is not None:
            lp[ok] = res[0]
            if need_grad:
                G[ok] = res[1]
        return lp, G

    def _log_prob_grad_rows(self, U, propto=True, need_grad=True, pre=None):
        """The in-support rows' (lp, grad), evaluating the likelihood at once."""
        gen = self._lpg_gen(U, propto, need_grad, pre)
        try:
            req = next(gen)
            gen.send(self._lik_rows(*req))
        except StopIteration as e:
            return e.value
        raise RuntimeError("internal: log-density generator did not finish")

    def _lpg_gen(self, U, propto=True, need_grad=True, pre=None):
        """Generator: yields the likelihood request (blens [m, B], model
        vectors [m, 10 + 2C]) of the draws that reach it, receives their output
        rows, returns (lp, grad) through StopIteration."""
        n = U.shape[0]
        sp = self.spec
        S, C = self.S, self.C
        vals, states, lp = self.constrain(U) if pre is None else pre
        lp = np.array(lp, np.float64)
        gx = {p.name: np.zeros((n,) + p.tr.shape) for p in self.params}

        # ---- substitution / site models
        freqs, R = self._q_params(vals, n)
        rs, ps = self._site_rates(vals, n)

        # ---- branch lengths
        if self.clock:
            h = self._heights(vals, n)
            span = self._span(h)
            mult, subs = self._multiplier(vals, n)
            blens = span * mult  # an overflow here is rejected just below
        else:
            blens = vals["blens"]

        # ---- likelihood (GPU); draws whose parameters over/underflowed in the
        # transforms are rejected without a launch (Stan: domain error)
        mv = np.concatenate([freqs, R, rs, ps], axis=1)
        ok = (np.isfinite(lp) & np.all(np.isfinite(mv), axis=1) & np.all(np.isfinite(blens), axis=1)
              & np.all(freqs > 0, axis=1))
        # compact output rows (include/phylo_hip.h): [ll, d/dblens, d/drs, d/dps,
        # d/dfreqs root term, d/d exchangeabilities, d/dfreqs]; zeros where not evaluated
        o = 1 + self.B + 2 * C
        rows = np.zeros((n, o + 14))
        rows[:, 0] = -np.inf
        if ok.any():
            sel = np.nonzero(ok)[0]
            got = yield (blens[sel], mv[sel])
            rows[sel] = got[:, :o + 14]
        ll = rows[:, 0]
        lp = lp + ll
        bad = ~np.isfinite(lp)

        # ---- priors (Stan ~ statements, constants dropped)
        if sp.categories > 1 and sp.heterogeneity == "weibull":
            lp = lp - vals["wshape"]
            gx["wshape"] -= 1.0
        if sp.model == "HKY":
            k = vals["kappa"]
            lk = np.log(k)
            lp = lp - lk - (lk - 1.0) ** 2 / (2.0 * 1.25 ** 2)
            gx["kappa"] += -1.0 / k - (lk - 1.0) / (1.25 ** 2 * k)
        g_h = None
        if self.clock:
            g_h = np.zeros((n, S - 1))
            g_subs_prior = g_span_prior = None
            if sp.estimate_rate and sp.clock == "strict":
                lp = lp - 1000.0 * vals["rate"]
                gx["rate"] -= 1000.0
            elif sp.relaxed:
                c_lp, g_subs_prior, g_span_prior, gh = clocks.clock_prior(self.ctree, sp.clock, vals, subs, span)
                lp = lp + c_lp
                for name, g in gh.items():
                    gx[name] += g
            if sp.speciation == "bd":
                b_lp, g_hb, g_a, g_r = clocks.birth_death(h, vals["netDiversificationRate"],
                                                          vals["relativeExtinctionRate"])
                lp = lp + b_lp
                g_h += g_hb
                gx["netDiversificationRate"] += g_a
                gx["relativeExtinctionRate"] += g_r
            # log-Jacobian of the height transform (generate_script.py:739-752)
            if self._nat is not None:
                jl = np.zeros(n)
                self._nat.jacobian(h, jl, g_h)
                lp = lp + jl
            else:
                nr = self.nonroot_int
                gap = h[:, self.parent[nr] - S] - self.lowers[nr]
                lp = lp + np.log(gap).sum(axis=1)
                np.add.at(g_h.T, self.parent[nr] - S, (1.0 / gap).T)
            # coalescent
            if sp.coalescent is not None:
                times = np.empty((n, 2 * S - 1))
                times[:, :S] = self.lowers[:S] if sp.heterochronous else 0.0
                times[:, S:] = h
                if sp.coalescent == "constant":
                    th = vals["theta"]
                    coal = hostlib.constant_coalescent if self._nat is not None else priors.constant_coalescent
                    c_lp, g_t, g_th = coal(times, self.times_internal, th)
                    lp = lp + c_lp - np.log(th)  # theta ~ oneOnX()
                    gx["theta"] += g_th - 1.0 / th
                else:
                    pop = vals["thetas"]
                    if sp.coalescent == "skyride":
                        c_lp, g_t, g_pop = priors.skyride_coalescent(times, self.times_internal, pop)
                    else:
                        grid = np.linspace(0.0, float(sp.cutoff), int(sp.grid))[1:]
                        c_lp, g_t, g_pop = priors.skygrid_coalescent(times, self.times_internal, pop, grid)
                    tau = vals["tau"]
                    m_lp, g_pop2, g_tau = priors.gmrf(pop, tau)
                    lp = lp + c_lp + m_lp + (0.001 - 1.0) * np.log(tau) - 0.001 * tau
                    gx["thetas"] += g_pop + g_pop2
                    gx["tau"] += g_tau + (0.001 - 1.0) / tau - 0.001
                g_h += g_t[:, S:]
        else:
            lp = lp - 10.0 * blens.sum(axis=1)
            gx["blens"] -= 10.0
        if not propto:
            lp = lp + self.const
        lp = np.where(bad, -np.inf, lp)
        if not need_grad:
            return lp, None

        # ---- likelihood gradient -> constrained parameters
        g_bl = rows[:, 1:1 + self.B]
        g_rs = rows[:, 1 + self.B:1 + self.B + C]
        g_ps = rows[:, 1 + self.B + C:o]
        if sp.model != "JC69":
            # the engine's chain rule through Q's eigendecomposition (include/phylo_hip.h)
            good = np.nonzero(~bad)[0]
            if len(good):
                gr = rows[good, o + 4:o + 10]
                gf = rows[good, o + 10:o + 14]
                gx["freqs"][good] += gf
                if sp.model == "GTR":
                    gx["rates"][good] += gr
                else:
                    gx["kappa"][good] += gr[:, 1] + gr[:, 4]  # kappa enters AG and CT
        self._site_rates_backward(vals, g_rs, g_ps, gx, rs, ps)
        if self.clock:
            gspan = g_bl * mult
            g_mult = g_bl * span
            if sp.relaxed:
                gspan = gspan + g_span_prior
                g_subs = clocks.blens_multiplier_backward(self.ctree, sp.clock, g_mult) + g_subs_prior
                if sp.clock in clocks.MRF:
                    g_d, g_rate = clocks.rates_from_deltas_backward(self.ctree, subs, g_subs)
                    gx["deltas"] += g_d
                    gx["rate"] += g_rate
                else:
                    gx["substrates"] += g_subs
            elif sp.estimate_rate:
                gx["rate"] += g_mult.sum(axis=1)
            if self._nat is not None:
                self._nat.span_back(gspan, g_h)
                self._nat.heights_back(vals["props"], h, g_h, gx["props"], gx["height"])
            else:
                np.add.at(g_h.T, self.b_parent, gspan.T)
                np.add.at(g_h.T, self.b_hidx[self.b_internal], -gspan[:, self.b_internal].T)
                # heights <- props, height (reverse of the level sweep)
                props = vals["props"]
                gprops = np.zeros_like(props)
                for nodes, pidx, jidx, low in reversed(self.levels):
                    gn = g_h[:, nodes - S]
                    gprops[:, jidx] += gn * (h[:, pidx] - low)
                    np.add.at(g_h.T, pidx, (gn * props[:, jidx]).T)
                gx["props"] += gprops
                gx["height"] += g_h[:, self.root - S]
        else:
            gx["blens"] += g_bl

        # ---- constrained -> unconstrained (+ log-Jacobian terms)
        G = np.zeros((n, self.dim))
        for p in self.params:
            G[:, p.sl] = p.tr.backward(states[p.name], gx[p.name], 1.0)
        G[bad] = 0.0
        G[~np.isfinite(G)] = 0.0
        return lp, G

    def _site_rates_backward(self, vals, g_rs, g_ps, gx, rs, ps):
        sp = self.spec
        C = self.C
        if sp.categories > 1 and sp.heterogeneity == "weibull":
            w = vals["wshape"]
            if sp.invariant:
                pinv = vals["pinv"]
                cat = C - 1
                i = np.arange(2, C + 1, dtype=np.float64)
                x = -np.log(1.0 - (2.0 * (i - 2) + 1.0) / (2.0 * cat))
                for d in range(len(w)):
                    g = np.power(x, 1.0 / w[d])
                    dg = g * np.log(x) * (-1.0 / (w[d] * w[d]))
                    pvar = 1.0 - pinv[d]
                    m = g.sum() * pvar / cat
                    dm_w = dg.sum() * pvar / cat
                    dm_p = -g.sum() / cat
                    drs_w = dg / m - g * dm_w / (m * m)
                    drs_p = -g * dm_p / (m * m)
                    gx["wshape"][d] += (g_rs[d, 1:] * drs_w).sum()
                    gx["pinv"][d] += (g_rs[d, 1:] * drs_p).sum() + g_ps[d, 0] - g_ps[d, 1:].sum() / cat
                return
            # models.weibull_site_rates_dshape, all draws at once
            x = self._wx[None, :]
            g = np.power(x, 1.0 / w[:, None])
            dg = g * np.log(x) * (-1.0 / (w * w))[:, None]
            m = g.mean(axis=1, keepdims=True)
            dm = dg.mean(axis=1, keepdims=True)
            gx["wshape"] += (g_rs * (dg / m - g * dm / (m * m))).sum(axis=1)
            return
        if sp.categories > 1:
            p_ = vals["ps"]
            ru = vals["rate_unscaled"]
            tot = (p_ * ru).sum(axis=1, keepdims=True)
            # rs = ru / tot
            gtot = -(g_rs * ru).sum(axis=1, keepdims=True) / tot ** 2
            gx["rate_unscaled"] += g_rs / tot + gtot * p_
            gx["ps"] += g_ps + gtot * ru
            return
        if sp.invariant:
            pinv = vals["pinv"]
            gx["pinv"] += g_rs[:, 1] / (1.0 - pinv) ** 2 + g_ps[:, 0] - g_ps[:, 1]

    # ------------------------------------------------------------ utilities
    def log_prob(self, U, propto=True):
        return self.log_prob_grad(U, propto=propto, need_grad=False)[0]

    def initial_point(self, rng, radius=2.0):
        """Stan's default initialisation: uniform(-2, 2) on the unconstrained scale."""
        return rng.uniform(-radius, radius, self.dim)

    def initialize(self, rng, radius=2.0, max_tries=100):
        """Stan ``services::util::initialize`` with random inits: up to 100
        uniform(-2, 2) draws until the log density and its gradient are both
        finite; the draw that passes is the initial point."""
        for _ in range(max_tries):
            q = self.initial_point(rng, radius)
            lp, G = self.log_prob_grad(q[None])
            if np.isfinite(lp[0]) and np.all(np.isfinite(G[0])):
                return q
        raise RuntimeError("Initialization failed after %d attempts: no random initial point with a finite log "
                           "density and gradient" % max_tries)

    def props_from_heights(self, heights):
        """Inverse of the height transform: ``props`` reproducing ``heights``
        (e.g. the input tree's, to start a chain there)."""
        h = np.asarray(heights, np.float64)
        props = np.empty(self.S - 2)
        for nodes, pidx, jidx, low in self.levels:
            props[jidx] = (h[nodes - self.S] - low) / (h[pidx] - low)
        return props

    def unconstrain(self, values):
        """dict name -> constrained value  ->  unconstrained vector."""
        u = np.zeros(self.dim)
        for p in self.params:
            u[p.sl] = p.tr.unconstrain(values[p.name])[0]
        return u

    def column_names(self):
        """Stan CSV column names of the parameters + transformed parameters."""
        names = []
        U0 = np.zeros((1, self.dim))
        for name, arr in self.transformed(U0):
            a = np.asarray(arr)
            if a.ndim == 1:
                names.append(name)
            else:
                names += ["%s.%d" % (name, k + 1) for k in range(a.shape[1])]
        return names

    def flat_rows(self, U):
        """[n, len(column_names())] constrained values of draws U."""
        cols = []
        for _, arr in self.transformed(U):
            a = np.asarray(arr, np.float64)
            cols.append(a[:, None] if a.ndim == 1 else a)
        return np.concatenate(cols, axis=1)
