"""ctypes binding of ``libphylo_host.so`` (csrc/host_model.cpp): native host
pieces of the clock models -- heights transform, log-Jacobian, branch spans
and the constant coalescent, with their reverse passes.

The numpy restatements in ``posterior.py`` / ``priors.py`` stay the
specification (``tests/test_hostlib.py`` compares the two); the posterior
uses this library when it is built, because these loops are the per-round
host cost of NUTS on a clock model.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PHYLO_HOST_LIB") or os.path.join(_HERE, "libphylo_host.so")
_lib = None

# every pointer is passed as an address (c_void_p): cheaper per call than
# typed ctypes pointers, which matters at one call per gradient round
_D = _I = _U8 = ctypes.c_void_p
_i = ctypes.c_int


def load():
    """The library, or None when it is not built."""
    global _lib
    if _lib is None and os.path.exists(LIB_PATH):
        lib = ctypes.CDLL(LIB_PATH)
        lib.phh_heights.argtypes = [_i, _i, _i, _I, _I, _I, _D, _i, _i, _D, _D, _D]
        lib.phh_heights_back.argtypes = [_i, _i, _i, _I, _I, _I, _D, _i, _i, _D, _D, _D, _D, _D]
        lib.phh_height_jacobian.argtypes = [_i, _i, _i, _I, _D, _D, _D, _D]
        lib.phh_span.argtypes = [_i, _i, _i, _I, _I, _D, _D, _D]
        lib.phh_span_back.argtypes = [_i, _i, _i, _I, _I, _D, _D]
        lib.phh_constant_coalescent.argtypes = [_i, _i, _D, _U8, _D, _D, _D, _D]
        for f in ("phh_heights", "phh_heights_back", "phh_height_jacobian", "phh_span", "phh_span_back",
                  "phh_constant_coalescent"):
            getattr(lib, f).restype = None
        if hasattr(lib, "phh_strict_create"):
            lib.phh_strict_create.argtypes = [_i, _i, _i, _i, _i, _i, ctypes.c_double, _i, _i, ctypes.c_double, _i,
                                              _I, _i, _I, _I, _I, _D, _i, _I, _I, _D, _i, _I, _D, _D]
            lib.phh_strict_create.restype = ctypes.c_void_p
            lib.phh_strict_free.argtypes = [ctypes.c_void_p]
            lib.phh_strict_free.restype = None
            lib.phh_strict_pre.argtypes = [ctypes.c_void_p, _i, _D, _D, _D, _I]
            lib.phh_strict_pre.restype = ctypes.c_int
            lib.phh_strict_post.argtypes = [ctypes.c_void_p, _i, _D, _D, _i, _I, _i, _D, _D]
            lib.phh_strict_post.restype = None
        if hasattr(lib, "phn_create"):
            _f = ctypes.c_double
            lib.phn_create.argtypes = [_i, _i, _D, _D, _i, _i, _i, _i, _f, _f, _f, _f, _f, _i, _i, _i, _f]
            lib.phn_create.restype = ctypes.c_void_p
            lib.phn_free.argtypes = [ctypes.c_void_p]
            lib.phn_free.restype = None
            lib.phn_step.argtypes = [ctypes.c_void_p, _i, _I, _D, _D, _D, _I]
            lib.phn_step.restype = ctypes.c_int
            lib.phn_error.argtypes = [ctypes.c_void_p, _i]
            lib.phn_error.restype = ctypes.c_int
            lib.phn_info.argtypes = [ctypes.c_void_p, _i, ctypes.POINTER(ctypes.c_long),
                                     ctypes.POINTER(ctypes.c_double), _D]
            lib.phn_info.restype = ctypes.c_int
            lib.phn_draws.argtypes = [ctypes.c_void_p, _i, _D, _D]
            lib.phn_draws.restype = None
        if hasattr(lib, "phn_set_static_hmc"):
            lib.phn_set_static_hmc.argtypes = [ctypes.c_void_p, ctypes.c_double]
            lib.phn_set_static_hmc.restype = None
        if hasattr(lib, "phn_run"):
            _p = ctypes.c_void_p
            lib.phn_run.argtypes = [_p, _p, _p, _p, _p, _i, _i, _i, _i, ctypes.POINTER(ctypes.c_long)]
            lib.phn_run.restype = ctypes.c_int
        _lib = lib
    return _lib


def _d(a):
    return a.ctypes.data


def _c(a, dtype=np.float64):
    return np.ascontiguousarray(a, dtype=dtype)


class ClockTreeNative:
    """Index arrays of one tree in the layout the native routines take."""

    def __init__(self, S, order_nodes, order_par, order_prop, order_low, root_h, b_parent, b_hidx, b_internal,
                 b_lower, jac_par, jac_low):
        self.lib = load()
        self.S = S
        self.H = S - 1
        self.np = S - 2
        self.node = _c(order_nodes, np.int32)
        self.par = _c(order_par, np.int32)
        self.prop = _c(order_prop, np.int32)
        self.low = _c(order_low)
        self.m = len(self.node)
        self.root = int(root_h)
        self.bpar = _c(b_parent, np.int32)
        self.bh = _c(np.where(b_internal, b_hidx, -1), np.int32)
        self.blow = _c(b_lower)
        self.B = len(self.bpar)
        self.jpar = _c(jac_par, np.int32)
        self.jlow = _c(jac_low)
        # addresses of the static index arrays, resolved once
        self.p_node, self.p_par, self.p_prop, self.p_low = (a.ctypes.data for a in (self.node, self.par, self.prop,
                                                                                      self.low))
        self.p_bpar, self.p_bh, self.p_blow = (a.ctypes.data for a in (self.bpar, self.bh, self.blow))
        self.p_jpar, self.p_jlow = self.jpar.ctypes.data, self.jlow.ctypes.data

    def heights(self, props, height):
        props, height = _c(props), _c(height)
        n = props.shape[0]
        h = np.empty((n, self.H))
        self.lib.phh_heights(n, self.H, self.m, self.p_node, self.p_par, self.p_prop, self.p_low, self.root, self.np,
                             _d(props), _d(height), _d(h))
        return h

    def heights_back(self, props, h, gh, gprops, gheight):
        """In place: consumes gh, accumulates gprops [n, S-2] and gheight [n]."""
        props, h = _c(props), _c(h)
        n = props.shape[0]
        self.lib.phh_heights_back(n, self.H, self.m, self.p_node, self.p_par, self.p_prop, self.p_low, self.root,
                                  self.np, _d(props), _d(h), _d(gh), _d(gprops), _d(gheight))

    def jacobian(self, h, lp, gh):
        h = _c(h)
        self.lib.phh_height_jacobian(h.shape[0], self.H, len(self.jpar), self.p_jpar, self.p_jlow, _d(h), _d(lp),
                                     _d(gh))

    def span(self, h):
        h = _c(h)
        out = np.empty((h.shape[0], self.B))
        self.lib.phh_span(h.shape[0], self.H, self.B, self.p_bpar, self.p_bh, self.p_blow, _d(h), _d(out))
        return out

    def span_back(self, gspan, gh):
        gspan = _c(gspan)
        self.lib.phh_span_back(gspan.shape[0], self.H, self.B, self.p_bpar, self.p_bh, _d(gspan), _d(gh))


class StrictPosterior:
    """The strict-clock log density + gradient around the likelihood in two
    native phases (csrc/host_model.cpp phh_strict_*): ``pre`` maps draws U to
    the branch lengths / model vectors of those that reach the likelihood,
    ``post`` maps the likelihood's rows to (lp, G).  ``posterior.Posterior``
    builds one for the specs it covers; its numpy path is the specification
    (tests/test_hostlib.py compares the two)."""

    def __init__(self, nat, S, B, C, model, weibull, est_rate, fixed_rate, coal, heterochronous, lower_root, dim,
                 offsets, lowers):
        self.lib = load()
        self.nat = nat  # keeps the index arrays alive
        self.B, self.C, self.dim = B, C, dim
        self.ml = 10 + 2 * C
        offs = _c(offsets, np.int32)
        self.lowers = _c(lowers)
        self.h = self.lib.phh_strict_create(
            S, B, C, model, int(weibull), int(est_rate), float(fixed_rate), int(coal), int(heterochronous),
            float(lower_root), dim, offs.ctypes.data, nat.m, nat.p_node, nat.p_par, nat.p_prop, nat.p_low, nat.root,
            nat.p_bpar, nat.p_bh, nat.p_blow, len(nat.jpar), nat.p_jpar, nat.p_jlow, self.lowers.ctypes.data)
        self._n = 0
        self._rowlen = 0
        self._last_u = None

    # Work arrays with their addresses resolved once (``ndarray.ctypes`` costs
    # ~2.5 us a call: nine of them were a fifth of a NUTS round's host time).
    # pre / post copy their operands in and their results out.
    def _buffers(self, n):
        if n > self._n:
            self._n = n
            self.U = np.empty((n, self.dim))
            self.blens = np.empty((n, self.B))
            self.mv = np.empty((n, self.ml))
            self.sel = np.empty(n, np.int32)
            self.psel = np.empty(n, np.int32)
            self.lp = np.empty(n)
            self.G = np.empty((n, self.dim))
            self.rows = np.empty((n, max(self._rowlen, 1)))
            self._p = {k: getattr(self, k).ctypes.data for k in ("U", "blens", "mv", "sel", "psel", "lp", "G", "rows")}
        return self._p

    def pre(self, U):
        """U [n, dim] -> (count, blens [count, B], model vectors [count, ml], sel [n])."""
        n = U.shape[0]
        p = self._buffers(n)
        self.U[:n] = U
        self._last_u = U
        cnt = self.lib.phh_strict_pre(self.h, n, p["U"], p["blens"], p["mv"], p["sel"])
        return cnt, self.blens[:cnt], self.mv[:cnt], self.sel[:n].copy()

    def post(self, U, rows, sel, need_grad=True):
        n = U.shape[0]
        p = self._buffers(n)
        if U is not self._last_u:  # pre's draws are in self.U already (the begin / end pair)
            self.U[:n] = U
            self._last_u = None
        rowlen = rows.shape[1] if rows is not None and len(rows) else 1
        if rowlen != self.rows.shape[1]:  # the row length is the stride phh_strict_post reads with
            self._rowlen = rowlen
            self.rows = np.empty((self._n, rowlen))
            p["rows"] = self.rows.ctypes.data
        if rows is not None and len(rows):
            self.rows[:len(rows)] = rows
        self.psel[:n] = sel
        self.lib.phh_strict_post(self.h, n, p["U"], p["rows"], rowlen, p["psel"], int(need_grad), p["lp"],
                                 p["G"] if need_grad else None)
        return self.lp[:n].copy(), (self.G[:n].copy() if need_grad else None)

    def __del__(self):
        if getattr(self, "h", None) and self.lib is not None:
            self.lib.phh_strict_free(self.h)
            self.h = None


def constant_coalescent(times, internal, theta):
    """Native ``priors.constant_coalescent``: (logP [n], dtimes [n, N], dtheta [n])."""
    lib = load()
    times = _c(times)
    n, N = times.shape
    intl = _c(internal, np.uint8)
    theta = _c(theta)
    lp = np.empty(n)
    g = np.empty((n, N))
    dth = np.empty(n)
    lib.phh_constant_coalescent(n, N, _d(times), intl.ctypes.data, _d(theta), _d(lp), _d(g), _d(dth))
    return lp, g, dth
