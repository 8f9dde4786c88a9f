"""Adaptive NUTS with a diagonal metric -- the sampler behind
``phylostan run -a nuts`` (``phylostan/phylostan.py:318-321``:
``sm.sampling(algorithm='NUTS', chains, iter, thin, seed)``).

Algorithm: Stan's ``adapt_diag_e_nuts`` (multinomial trajectory sampling
with the across-subtree no-U-turn checks of ``base_nuts::transition`` /
``build_tree``; leapfrog ``expl_leapfrog``; Nesterov dual-averaging step
size, delta 0.8, gamma 0.05, kappa 0.75, t0 10; windowed variance
adaptation, init buffer 75, term buffer 50, base window 25, regularised
``n/(n+5) var + 1e-3 * 5/(n+5)``; ``init_stepsize`` doubling/halving;
max tree depth 10; max Delta-H 1000).  Stan's boost RNG streams are not
reproduced (numpy PCG64 per chain).

MI355X shape: every chain is a *coroutine* that yields the positions whose
log density and gradient it needs; ``run_chains`` advances all chains in
lockstep and evaluates the pending positions of all of them in ONE batched
call (one GPU launch of ``n_chains`` draws), so 8 chains cost about as much
wall time per leapfrog step as one.

The generators below are the specification.  ``run_chains`` runs the same
programs natively by default (csrc/nuts_host.cpp: a state machine per chain
drawing from the chains' numpy Generators, bitwise these chains' draws up to
15 dimensions), and for the strict-clock posterior around a TreeLikelihood
the whole round loop too (``phn_run``: no Python per gradient round).
"""
import ctypes
import math
import os
import time

import numpy as np


def _sdot(a, b):
    """sum_i a_i b_i as one sequential sum of rounded products: numpy's
    add.accumulate is a strict left-to-right loop (np.dot's order depends on
    the BLAS build and the CPU), so csrc/nuts_host.cpp's dot reproduces it
    bit for bit on any host."""
    if len(a) == 0:
        return 0.0
    return float(np.cumsum(np.multiply(a, b))[-1])


def _log_sum_exp(a, b):
    if a == -math.inf:
        return b
    if b == -math.inf:
        return a
    m = max(a, b)
    return m + math.log(math.exp(a - m) + math.exp(b - m))


class _Point:
    __slots__ = ("q", "p", "lp", "g")

    def __init__(self, q, p, lp, g):
        self.q, self.p, self.lp, self.g = q, p, lp, g

    def copy(self):
        # shallow: the sampler never changes a position, momentum or gradient
        # array in place (every update binds a new array), so a snapshot can
        # share them
        return _Point(self.q, self.p, self.lp, self.g)


class Chain:
    """One NUTS chain as a generator (``program()``): it yields a position
    ``q`` and expects ``(lp, grad)`` sent back; it records its draws."""

    def __init__(self, dim, q0, rng, num_warmup=1000, num_samples=1000, thin=1, max_depth=10,
                 delta=0.8, gamma=0.05, kappa=0.75, t0=10.0, stepsize=1.0, init_buffer=75,
                 term_buffer=50, base_window=25, max_delta_h=1000.0):
        self.dim = dim
        self.q0 = np.asarray(q0, np.float64).copy()
        self.rng = rng
        self.num_warmup = int(num_warmup)
        self.num_samples = int(num_samples)
        self.thin = max(1, int(thin))
        self.max_depth = max_depth
        self.delta, self.gamma, self.kappa, self.t0 = delta, gamma, kappa, t0
        self.eps = float(stepsize)
        self.max_delta_h = max_delta_h
        self.inv_metric = np.ones(dim)
        self._setup_windows(init_buffer, term_buffer, base_window)
        self.draws = []  # (q, lp, accept, eps, depth, n_leapfrog, divergent, energy, warmup)
        self.n_grad = 0

    # -------------------------------------------------------- adaptation
    def _setup_windows(self, init_buffer, term_buffer, base_window):
        W = self.num_warmup
        if W < 20:
            self.adapt_init, self.adapt_term, self.adapt_base = W, 0, 0
            self.windows = False
            return
        self.windows = True
        if init_buffer + base_window + term_buffer > W:
            init_buffer = int(0.15 * W)
            term_buffer = int(0.1 * W)
            base_window = W - (init_buffer + term_buffer)
        self.adapt_init, self.adapt_term, self.adapt_base = init_buffer, term_buffer, base_window
        self.win_counter = 0
        self.win_size = base_window
        self.next_window = init_buffer + base_window - 1
        self._w_n = 0
        self._w_mean = np.zeros(self.dim)
        self._w_m2 = np.zeros(self.dim)

    def _in_window(self):
        W = self.num_warmup
        return self.adapt_init <= self.win_counter < W - self.adapt_term and self.win_counter != W

    def _end_window(self):
        return self.win_counter == self.next_window and self.win_counter != self.num_warmup

    def _compute_next_window(self):
        W, term = self.num_warmup, self.adapt_term
        if self.next_window == W - term - 1:
            return
        self.win_size *= 2
        self.next_window = self.win_counter + self.win_size
        if self.next_window != W - term - 1:
            if self.next_window + 2 * self.win_size >= W - term:
                self.next_window = W - term - 1

    def _learn_variance(self, q):
        if not self.windows:
            return False
        if self._in_window():
            self._w_n += 1
            d = q - self._w_mean
            self._w_mean += d / self._w_n
            self._w_m2 += d * (q - self._w_mean)
        if self._end_window():
            self._compute_next_window()
            n = float(self._w_n)
            var = self._w_m2 / (n - 1.0) if n > 1 else np.ones(self.dim)
            self.inv_metric = (n / (n + 5.0)) * var + 1e-3 * (5.0 / (n + 5.0))
            self._w_n = 0
            self._w_mean[:] = 0.0
            self._w_m2[:] = 0.0
            self.win_counter += 1
            return True
        self.win_counter += 1
        return False

    def _da_restart(self):
        self.da_counter = 0
        self.s_bar = 0.0
        self.x_bar = 0.0
        self.mu = math.log(10.0 * self.eps)

    def _learn_stepsize(self, adapt_stat):
        self.da_counter += 1
        adapt_stat = min(1.0, adapt_stat)
        eta = 1.0 / (self.da_counter + self.t0)
        self.s_bar = (1.0 - eta) * self.s_bar + eta * (self.delta - adapt_stat)
        x = self.mu - self.s_bar * math.sqrt(self.da_counter) / self.gamma
        x_eta = self.da_counter ** (-self.kappa)
        self.x_bar = (1.0 - x_eta) * self.x_bar + x_eta * x
        self.eps = math.exp(x)

    # ------------------------------------------------------ hamiltonian
    def _sample_p(self):
        return self.rng.standard_normal(self.dim) / np.sqrt(self.inv_metric)

    def _H(self, z):
        if not np.isfinite(z.lp):
            return math.inf
        return -z.lp + 0.5 * _sdot(self.inv_metric * z.p, z.p)

    def _evolve(self, z, eps):
        """expl_leapfrog: one step in place; yields the new q for (lp, grad)."""
        z.p = z.p + 0.5 * eps * z.g
        z.q = z.q + eps * self.inv_metric * z.p
        lp, g = yield z.q
        self.n_grad += 1
        z.lp = lp
        z.g = g if np.all(np.isfinite(g)) else np.zeros_like(z.q)
        if not np.isfinite(lp):
            z.lp = -math.inf
        z.p = z.p + 0.5 * eps * z.g

    def _init_stepsize(self, z0):
        if self.eps == 0 or self.eps > 1e7 or math.isnan(self.eps):
            return
        z = z0.copy()
        z.p = self._sample_p()
        H0 = self._H(z)
        yield from self._evolve(z, self.eps)
        h = self._H(z)
        dH = H0 - (math.inf if math.isnan(h) else h)
        direction = 1 if dH > math.log(0.8) else -1
        while True:
            z = z0.copy()
            z.p = self._sample_p()
            H0 = self._H(z)
            yield from self._evolve(z, self.eps)
            h = self._H(z)
            dH = H0 - (math.inf if math.isnan(h) else h)
            if direction == 1 and not dH > math.log(0.8):
                break
            if direction == -1 and not dH < math.log(0.8):
                break
            self.eps = self.eps * 2.0 if direction == 1 else self.eps * 0.5
            if self.eps > 1e7:
                raise RuntimeError("NUTS: posterior is improper (step size > 1e7)")
            if self.eps == 0:
                raise RuntimeError("NUTS: no acceptable small step size")

    @staticmethod
    def _criterion(ps_minus, ps_plus, rho):
        return _sdot(ps_plus, rho) > 0 and _sdot(ps_minus, rho) > 0

    def _build_tree(self, depth, z, H0, sign, st):
        """Returns (valid, z_propose, p_sharp_beg, p_sharp_end, rho, p_beg,
        p_end, log_sum_weight); ``st`` carries n_leapfrog, sum_metro_prob,
        divergent.  ``z`` is advanced in place."""
        if depth == 0:
            yield from self._evolve(z, sign * self.eps)
            st["n_leapfrog"] += 1
            h = self._H(z)
            if math.isnan(h):
                h = math.inf
            if h - H0 > self.max_delta_h:
                st["divergent"] = True
            lsw = H0 - h if h != math.inf else -math.inf
            st["sum_metro_prob"] += 1.0 if H0 - h > 0 else math.exp(H0 - h)
            ps = self.inv_metric * z.p
            return (not st["divergent"], z.copy(), ps, ps, z.p, z.p, z.p, lsw)
        v1, zp, ps_beg, ps_init_end, rho_init, p_beg, p_init_end, lsw_init = \
            yield from self._build_tree(depth - 1, z, H0, sign, st)
        if not v1:
            return (False, zp, ps_beg, ps_init_end, rho_init, p_beg, p_init_end, lsw_init)
        v2, zp_final, ps_final_beg, ps_end, rho_final, p_final_beg, p_end, lsw_final = \
            yield from self._build_tree(depth - 1, z, H0, sign, st)
        if not v2:
            return (False, zp, ps_beg, ps_end, rho_init, p_beg, p_end, lsw_init)
        lsw_sub = _log_sum_exp(lsw_init, lsw_final)
        if lsw_final > lsw_sub:
            zp = zp_final
        else:
            if self.rng.uniform() < math.exp(lsw_final - lsw_sub):
                zp = zp_final
        rho_sub = rho_init + rho_final
        ok = self._criterion(ps_beg, ps_end, rho_sub)
        ok &= self._criterion(ps_beg, ps_final_beg, rho_init + p_final_beg)
        ok &= self._criterion(ps_init_end, ps_end, rho_final + p_init_end)
        return (ok, zp, ps_beg, ps_end, rho_sub, p_beg, p_end, lsw_sub)

    def _transition(self, z0):
        z = z0.copy()
        z.p = self._sample_p()
        H0 = self._H(z)
        z_fwd, z_bck, z_sample = z.copy(), z.copy(), z.copy()
        ps0 = self.inv_metric * z.p
        p_fwd_fwd = p_fwd_bck = p_bck_fwd = p_bck_bck = rho = z.p
        ps_fwd_fwd = ps_fwd_bck = ps_bck_fwd = ps_bck_bck = ps0
        lsw = 0.0
        st = {"n_leapfrog": 0, "sum_metro_prob": 0.0, "divergent": False}
        depth = 0
        while depth < self.max_depth:
            if self.rng.uniform() > 0.5:
                rho_bck = rho
                p_bck_fwd, ps_bck_fwd = p_fwd_bck, ps_fwd_bck
                zz = z_fwd
                valid, zp, ps_fwd_bck, ps_fwd_fwd, rho_fwd, p_fwd_bck, p_fwd_fwd, lsw_sub = \
                    yield from self._build_tree(depth, zz, H0, 1.0, st)
                z_fwd = zz
            else:
                rho_fwd = rho
                p_fwd_bck, ps_fwd_bck = p_bck_fwd, ps_bck_fwd
                zz = z_bck
                valid, zp, ps_bck_fwd, ps_bck_bck, rho_bck, p_bck_fwd, p_bck_bck, lsw_sub = \
                    yield from self._build_tree(depth, zz, H0, -1.0, st)
                z_bck = zz
            if not valid:
                break
            depth += 1
            if lsw_sub > lsw:
                z_sample = zp
            elif self.rng.uniform() < math.exp(lsw_sub - lsw):
                z_sample = zp
            lsw = _log_sum_exp(lsw, lsw_sub)
            rho = rho_bck + rho_fwd
            ok = self._criterion(ps_bck_bck, ps_fwd_fwd, rho)
            ok &= self._criterion(ps_bck_bck, ps_fwd_bck, rho_bck + p_fwd_bck)
            ok &= self._criterion(ps_bck_fwd, ps_fwd_fwd, rho_fwd + p_bck_fwd)
            if not ok:
                break
        n_lf = st["n_leapfrog"]
        accept = st["sum_metro_prob"] / max(n_lf, 1)
        energy = self._H(z_sample)
        return z_sample, accept, depth, n_lf, st["divergent"], energy

    # ----------------------------------------------------------- program
    def program(self):
        lp, g = yield self.q0
        z = _Point(self.q0.copy(), np.zeros(self.dim), lp, g)
        if not np.isfinite(lp):
            raise RuntimeError("NUTS: initial point has non-finite log density")
        yield from self._init_stepsize(z)
        self._da_restart()
        total = self.num_warmup + self.num_samples
        for it in range(total):
            warm = it < self.num_warmup
            eps_used = self.eps
            z_new, accept, depth, n_lf, div, energy = yield from self._transition(z)
            z = _Point(z_new.q, np.zeros(self.dim), z_new.lp, z_new.g)
            if warm:
                self._learn_stepsize(accept)
                if self._learn_variance(z.q):
                    yield from self._init_stepsize(z)
                    self._da_restart()
                if it == self.num_warmup - 1:
                    self.eps = math.exp(self.x_bar)  # complete_adaptation
            if it % self.thin == 0:
                self.draws.append((z.q.copy(), z.lp, accept, eps_used, depth, n_lf, int(div), energy, warm))
        return self


class StaticHMCChain(Chain):
    """Stan's ``adapt_diag_e_static_hmc`` (``sm.sampling(algorithm='HMC')``,
    phylostan.py:319-321): a fixed integration time T (``int_time``, Stan's
    default 2 pi) covered by L = max(1, int(T / eps)) leapfrog steps, one
    Metropolis accept/reject of the end point (accept_stat = min(1,
    exp(H0 - h)), NaN energy = rejection), and the same step-size and
    diagonal-metric adaptation as NUTS (after every adaptation update L is
    recomputed from the nominal step size; ``init_stepsize`` leaves it
    alone, as ``base_hmc::init_stepsize`` does).  The draw record keeps the
    NUTS layout with int_time in the tree-depth slot and divergent = 0."""

    def __init__(self, dim, q0, rng, num_warmup=1000, num_samples=1000, thin=1, int_time=2 * math.pi, **kw):
        kw.pop("max_depth", None)
        super().__init__(dim, q0, rng, num_warmup, num_samples, thin, **kw)
        self.T = float(int_time)
        self._update_L()

    def _update_L(self):
        self.L = max(1, int(self.T / self.eps))

    def _transition(self, z0):
        z = z0.copy()
        z.p = self._sample_p()
        z_init = z.copy()
        H0 = self._H(z)
        n_lf = self.L
        for _ in range(n_lf):
            yield from self._evolve(z, self.eps)
        h = self._H(z)
        if math.isnan(h):
            h = math.inf
        # Stan: accept_prob = exp(H0 - h) (inf when the energy drops by more
        # than ~709 nats, i.e. accepted); math.exp would overflow there
        accept = 0.0 if h == math.inf else (1.0 if H0 - h > 0 else math.exp(H0 - h))
        if accept < 1.0 and self.rng.uniform() > accept:
            z = z_init
        accept = min(1.0, accept)
        return z, accept, self.T, n_lf, False, self._H(z)

    def program(self):
        lp, g = yield self.q0
        z = _Point(self.q0.copy(), np.zeros(self.dim), lp, g)
        if not np.isfinite(lp):
            raise RuntimeError("HMC: initial point has non-finite log density")
        yield from self._init_stepsize(z)
        self._da_restart()
        total = self.num_warmup + self.num_samples
        for it in range(total):
            warm = it < self.num_warmup
            eps_used = self.eps
            z_new, accept, int_time, n_lf, div, energy = yield from self._transition(z)
            z = _Point(z_new.q, np.zeros(self.dim), z_new.lp, z_new.g)
            if warm:
                self._learn_stepsize(accept)
                self._update_L()
                if self._learn_variance(z.q):
                    yield from self._init_stepsize(z)
                    self._update_L()
                    self._da_restart()
                if it == self.num_warmup - 1:
                    # disengage_adaptation -> complete_adaptation(nom_epsilon) only:
                    # sampling keeps the L of the last warmup update, as Stan's
                    # adapt_diag_e_static_hmc does (no update_L_ there)
                    self.eps = math.exp(self.x_bar)
            if it % self.thin == 0:
                self.draws.append((z.q.copy(), z.lp, accept, eps_used, int_time, n_lf, 0, energy, warm))
        return self


_CHAIN_OPTIONS = dict(delta=0.8, gamma=0.05, kappa=0.75, t0=10.0, stepsize=1.0, init_buffer=75, term_buffer=50,
                      base_window=25, max_delta_h=1000.0)  # Chain.__init__'s defaults


class NativeChain:
    """A finished chain of the native sampler, with ``Chain``'s result
    attributes (draws, n_grad, eps, inv_metric)."""

    def __init__(self, dim, draws, n_grad, eps, inv_metric):
        self.dim, self.draws, self.n_grad, self.eps, self.inv_metric = dim, draws, n_grad, eps, inv_metric


def native_available():
    from . import hostlib
    lib = hostlib.load()
    return lib if lib is not None and hasattr(lib, "phn_create") else None


def _run_native(lib, posterior, q0s, seeds, num_warmup, num_samples, thin, progress, max_depth, hmc=False, **kw):
    """``Chain`` (or, hmc=True, ``StaticHMCChain``) programs run by
    csrc/nuts_host.cpp (the same algorithm and random streams;
    tests/test_nuts_native.py): one C call per gradient round advances every
    chain and returns the positions of the next batched
    ``posterior.log_prob_grad`` call."""
    int_time = float(kw.pop("int_time", 2 * math.pi)) if hmc else None
    bad = set(kw) - set(_CHAIN_OPTIONS)
    if bad:
        raise TypeError("unexpected %s option(s) %s" % ("HMC" if hmc else "NUTS", sorted(bad)))
    o = dict(_CHAIN_OPTIONS, **kw)
    dim, n = posterior.dim, len(q0s)
    rngs = [np.random.default_rng(sd) for sd in seeds]  # alive while the chains draw from them
    bitgens = np.array([r.bit_generator.ctypes.bit_generator.value for r in rngs], np.uintp)
    q0 = np.ascontiguousarray(np.stack([np.asarray(q, np.float64).reshape(dim) for q in q0s]))
    h = lib.phn_create(n, dim, q0.ctypes.data, bitgens.ctypes.data, int(num_warmup), int(num_samples), int(thin),
                       int(max_depth), float(o["delta"]), float(o["gamma"]), float(o["kappa"]), float(o["t0"]),
                       float(o["stepsize"]), int(o["init_buffer"]), int(o["term_buffer"]), int(o["base_window"]),
                       float(o["max_delta_h"]))
    if hmc:
        lib.phn_set_static_hmc(h, int_time)
    try:
        native_loop = _native_loop_args(posterior, n)
        if native_loop is not None:  # every round in C++ (phn_run)
            rounds, t0 = ctypes.c_long(0), time.time()
            while True:
                r = lib.phn_run(h, *native_loop, 2000, ctypes.byref(rounds))
                if r <= 0:
                    break
                if progress:
                    nd = lib.phn_info(h, 0, None, None, None)
                    progress("NUTS: %d gradient rounds, %d draws (chain 0), %.1f s" % (rounds.value, nd, time.time() - t0))
            if r <= -1000000:
                from . import _lib
                _lib.check(-(r + 1000000), "phy_eval_submit / phy_eval_wait (native NUTS loop)")
            m = r
        else:
            m = _python_rounds(lib, h, posterior, n, dim, progress)
        if m < 0:
            code = lib.phn_error(h, -m - 1)
            raise RuntimeError({1: "%s: initial point has non-finite log density" % ("HMC" if hmc else "NUTS"),
                                2: "NUTS: posterior is improper (step size > 1e7)",
                                3: "NUTS: no acceptable small step size"}.get(code, "NUTS: chain failed (%d)" % code))
        out = []
        for c in range(n):
            ng, eps = ctypes.c_long(), ctypes.c_double()
            im = np.empty(dim)
            nd = lib.phn_info(h, c, ctypes.byref(ng), ctypes.byref(eps), im.ctypes.data)
            q, st = np.empty((nd, dim)), np.empty((nd, 8))
            lib.phn_draws(h, c, q.ctypes.data, st.ctypes.data)
            slot3 = float if hmc else int  # HMC: the integration time in the tree-depth slot
            draws = [(q[k], float(s[0]), float(s[1]), float(s[2]), slot3(s[3]), int(s[4]), int(s[5]), float(s[6]),
                      bool(s[7])) for k, s in enumerate(st)]
            out.append(NativeChain(dim, draws, int(ng.value), float(eps.value), im))
        return out
    finally:
        lib.phn_free(h)


def _native_loop_args(posterior, n):
    """phn_run's arguments after the sampler handle when the whole round can
    run natively -- the posterior's strict-clock native phases
    (hostlib.StrictPosterior) around a TreeLikelihood context whose
    phy_eval_submit takes all chains at once (n <= max_draws, n <= 128) --
    else None (the rounds go through Posterior.log_prob_grad).
    ``PHYLO_NUTS_LOOP=python`` forces the latter."""
    fast, lik = getattr(posterior, "_fast", None), getattr(posterior, "lik", None)
    if os.environ.get("PHYLO_NUTS_LOOP") == "python" or fast is None or lik is None:
        return None
    native = getattr(lik, "native_submit_wait", None)
    if native is None:
        return None
    sw = native(n)
    if sw is None:
        return None
    ctx, submit, wait, rowlen = sw
    return (ctypes.c_void_p(fast.h), ctypes.c_void_p(ctx), ctypes.c_void_p(submit), ctypes.c_void_p(wait),
            fast.B, fast.ml, rowlen)


def _python_rounds(lib, h, posterior, n, dim, progress):
    """The rounds through Posterior.log_prob_grad (any posterior and
    likelihood): one phn_step per round.  Returns phn_step's last result
    (0, or -(1 + chain) on a chain failure)."""
    # the round's arrays, addresses resolved once (ndarray.ctypes ~2.5 us)
    Q, LP, GR = np.empty((n, dim)), np.empty(n), np.empty((n, dim))
    idx_a, idx_b = np.empty(n, np.int32), np.empty(n, np.int32)
    pQ, pLP, pGR = Q.ctypes.data, LP.ctypes.data, GR.ctypes.data
    pa, pb = idx_a.ctypes.data, idx_b.ctypes.data
    m = lib.phn_step(h, 0, None, None, None, pQ, pa)
    rounds, t0 = 0, time.time()
    while m > 0:
        lp, G = posterior.log_prob_grad(Q[:m])
        LP[:m] = lp
        GR[:m] = G
        pa, pb = pb, pa
        m = lib.phn_step(h, m, pb, pLP, pGR, pQ, pa)
        rounds += 1
        if progress and rounds % 2000 == 0:
            nd = lib.phn_info(h, 0, None, None, None)
            progress("NUTS: %d gradient rounds, %d draws (chain 0), %.1f s" % (rounds, nd, time.time() - t0))
    return m


def run_chains(posterior, q0s, seeds, num_warmup=1000, num_samples=1000, thin=1, progress=None,
               max_depth=10, algorithm="nuts", native=None, **kw):
    """Run ``len(q0s)`` NUTS (or static HMC) chains in lockstep, batching
    every round of gradient requests into one ``posterior.log_prob_grad``
    call (one small-batch likelihood launch for all chains).  Every chain
    sees exactly the values it would see alone: evaluations are per draw,
    independent of the batch.  (Pipelining chain groups over two contexts
    was measured slower -- the host's cost is per call -- and retired.)

    NUTS runs on the native chains (csrc/nuts_host.cpp) when libphylo_host.so
    has them, unless ``native=False`` or ``PHYLO_NUTS=python``; the
    generators below are their specification."""
    dim = posterior.dim
    if native is None:
        native = os.environ.get("PHYLO_NUTS", "native") != "python"
    lib = native_available() if native else None
    if lib is not None and algorithm == "hmc" and not hasattr(lib, "phn_set_static_hmc"):
        lib = None
    if native and lib is None and os.environ.get("PHYLO_NUTS") == "native":
        raise RuntimeError("PHYLO_NUTS=native but libphylo_host.so has no native chains (run build())")
    if lib is not None:
        if algorithm == "hmc":
            kw.pop("max_depth", None)
        return _run_native(lib, posterior, q0s, seeds, num_warmup, num_samples, thin, progress, max_depth,
                           hmc=algorithm == "hmc", **kw)
    if algorithm == "hmc":
        chains = [StaticHMCChain(dim, q0, np.random.default_rng(sd), num_warmup, num_samples, thin, **kw)
                  for q0, sd in zip(q0s, seeds)]
    else:
        chains = [Chain(dim, q0, np.random.default_rng(sd), num_warmup, num_samples, thin,
                        max_depth=max_depth, **kw) for q0, sd in zip(q0s, seeds)]
    gens = [c.program() for c in chains]
    pending = {}
    for i, g in enumerate(gens):
        pending[i] = next(g)
    rounds = 0
    t0 = time.time()
    while pending:
        idx = list(pending)
        lp, G = posterior.log_prob_grad(np.stack([pending[i] for i in idx]))
        for j, i in enumerate(idx):
            try:
                pending[i] = gens[i].send((float(lp[j]), G[j]))
            except StopIteration:
                del pending[i]
        rounds += 1
        if progress and rounds % 2000 == 0:
            progress("%s: %d gradient rounds, %d draws (chain 0), %.1f s"
                     % (algorithm.upper(), rounds, len(chains[0].draws), time.time() - t0))
    return chains
