"""Host-side mirror of the reference's likelihood interface over the C-ABI.

In phylostan the likelihood is reached two ways, both replaced here:

* the emitted Stan model block -- data dict ``{peel, tipdata, weights, C,
  map, ...}`` (``phylostan/phylostan.py:181-286``) and parameters; the model
  block computes ``pmats`` (``generate_script.py:1425/1439/1447``) then
  ``target += log(sum(probs)) * weights[i]`` (``:961-1055``), and Stan's
  autodiff supplies the gradient;
* the external-function plugin ``real pruning_loglik(vector blens)``
  (``eigen/example.stan:3``, ``eigen/prune_stan.hpp:9-17``) returning the
  value and ``precomputed_gradients``.

``TreeLikelihood`` owns one ``phy_ctx`` (one GPU, one process); its
``log_prob`` / ``pruning_loglik`` return the value and the gradient the
Stan model would have produced.  There is no CPU fallback: without the HIP
library ``_lib.load()`` raises.
"""
import ctypes

import numpy as np

from . import _lib
from . import models


class EvalResult:
    """Unpacked output vector of one draw (layout: include/phylo_hip.h)."""

    __slots__ = ("loglik", "grad_blens", "grad_rs", "grad_ps", "grad_freq_root", "grad_rates", "grad_freqs",
                 "dLdP", "site_ll")

    def __init__(self, vec, B, C, site_ll=None):
        o = 1 + B + 2 * C
        og = o + 4 + 10
        self.loglik = float(vec[0])
        self.grad_blens = vec[1:1 + B].copy()
        self.grad_rs = vec[1 + B:1 + B + C].copy()
        self.grad_ps = vec[1 + B + C:o].copy()
        self.grad_freq_root = vec[o:o + 4].copy()
        self.grad_rates = vec[o + 4:o + 10].copy()   # d/d exchangeabilities AC AG AT CG CT GT
        self.grad_freqs = vec[o + 10:og].copy()      # d/d freqs: through Q plus the root term
        self.dLdP = vec[og:og + C * B * 16].reshape(C, B, 4, 4).copy() if len(vec) >= og + C * B * 16 else None
        self.site_ll = site_ll

    def as_dict(self):
        return {k: getattr(self, k) for k in self.__slots__}


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class TreeLikelihood:
    """GPU pruning likelihood of one alignment + topology.

    Parameters
    ----------
    tipcodes : uint8 [S, P] state masks (A=1, C=2, G=4, T=8, other 15)
    weights  : [P] pattern multiplicities
    peel0    : int [S-1, 3] 0-based peel rows (child1, child2, parent)
    rooted   : True for the clock (rooted) model variants
    model    : "JC69" | "HKY" | "GTR"
    C        : rate categories
    max_draws: parameter points per batched evaluation
    device   : HIP device ordinal
    devices  : a list of device ordinals -> ONE context over len(devices)
               contiguous pattern shards (phy_create_multi: every shard on
               its device, one reduction of the output rows per evaluation --
               RCCL all-reduce over distinct devices, a device-side sum when
               they are all the same)
    """

    _pending = 0  # draws of a submit_rows not yet collected

    def __init__(self, tipcodes, weights, peel0, rooted, model, C, max_draws=1, device=0, devices=None):
        self.lib = _lib.load()
        tipcodes = np.ascontiguousarray(tipcodes, dtype=np.uint8)
        self.S, self.P = tipcodes.shape
        self.C = int(C)
        self.rooted = bool(rooted)
        self.model = models.MODEL_IDS[model] if isinstance(model, str) else int(model)
        self.max_draws = int(max_draws)
        w = np.ascontiguousarray(weights, dtype=np.float64)
        peel = np.ascontiguousarray(peel0, dtype=np.int32)
        if w.shape != (self.P,):
            raise ValueError("weights must have shape (P,)")
        if peel.shape != (self.S - 1, 3):
            raise ValueError("peel must have shape (S-1, 3)")
        ctx = ctypes.c_void_p()
        if devices is not None:
            devs = np.ascontiguousarray(devices, dtype=np.int32)
            _lib.check(self.lib.phy_create_multi(self.S, self.P, self.C, int(self.rooted), self.model,
                                                 _ptr(tipcodes), _ptr(w), _ptr(peel), self.max_draws,
                                                 int(devs.size), _ptr(devs), ctypes.byref(ctx)), "phy_create_multi")
        else:
            _lib.check(self.lib.phy_create(self.S, self.P, self.C, int(self.rooted), self.model,
                                           _ptr(tipcodes), _ptr(w), _ptr(peel), self.max_draws,
                                           int(device), ctypes.byref(ctx)), "phy_create")
        self.ctx = ctx
        self.B = self.lib.phy_num_branches(ctx)
        self.outlen = self.lib.phy_output_len(ctx)
        self.model_len = 10 + 2 * self.C

    @classmethod
    def from_data(cls, data, model, C, **kw):
        """From a ``phylostan_amd.data.PhyloData`` (what ``phylostan run``
        builds before handing the dict to Stan)."""
        return cls(data.tipcodes, data.weights, data.peel0, data.rooted, model, C, **kw)

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.phy_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def program_info(self):
        vals = [ctypes.c_int() for _ in range(4)]
        _lib.check(self.lib.phy_program_info(self.ctx, *[ctypes.byref(v) for v in vals]),
                   "phy_program_info")
        return dict(zip(("nsteps", "nslots", "depth", "nblocks"), [v.value for v in vals]))

    def model_vector(self, freqs, rates, rs, ps):
        v = models.model_vector(freqs, rates, rs, ps)
        if v.shape != (self.model_len,):
            raise ValueError("model vector must have length 10 + 2C")
        return v

    def evaluate_batch(self, blens, model_vecs, site_ll=False):
        """n draws: blens [n, B], model_vecs [n, 10+2C] -> list of EvalResult."""
        blens = np.ascontiguousarray(np.atleast_2d(blens), dtype=np.float64)
        mv = np.ascontiguousarray(np.atleast_2d(model_vecs), dtype=np.float64)
        n = blens.shape[0]
        if blens.shape != (n, self.B) or mv.shape != (n, self.model_len):
            raise ValueError("bad shapes: blens %s model %s" % (blens.shape, mv.shape))
        out = np.empty((n, self.outlen))
        sl = np.empty((n, self.P)) if site_ll else None
        _lib.check(self.lib.phy_eval(self.ctx, n, _ptr(blens), _ptr(mv), _ptr(out),
                                     _ptr(sl) if site_ll else None), "phy_eval")
        return [EvalResult(out[k], self.B, self.C, sl[k] if site_ll else None) for k in range(n)]

    def evaluate_rows(self, blens, model_vecs):
        """n draws -> the raw output rows [n, outlen] (no per-draw objects:
        the sampler's path)."""
        blens, mv = np.asarray(blens, np.float64), np.asarray(model_vecs, np.float64)
        if blens.ndim == 1:
            blens, mv = blens[None], mv.reshape(1, -1)
        n = blens.shape[0]
        if blens.shape != (n, self.B) or mv.shape != (n, self.model_len):
            raise ValueError("bad shapes: blens %s model %s" % (blens.shape, mv.shape))
        if n <= min(self.max_draws, self._STAGE_DRAWS):  # a sampler's call: the staging arrays
            sbl, smv, sout, pbl, pmv, pout = self._stage()
            sbl[:n] = blens
            smv[:n] = mv
            _lib.check(self.lib.phy_eval(self.ctx, n, pbl, pmv, pout, None), "phy_eval")
            return sout[:n].copy()
        blens, mv = np.ascontiguousarray(blens), np.ascontiguousarray(mv)
        out = np.empty((n, self.outlen))
        _lib.check(self.lib.phy_eval(self.ctx, n, blens.ctypes.data, mv.ctypes.data, out.ctypes.data, None),
                   "phy_eval")
        return out

    _STAGE_DRAWS = 128  # phy_eval_submit's batch limit (PIN_DRAWS)

    def _stage(self):
        """Host staging arrays of the submit / wait pair with their addresses
        resolved once: ``ndarray.ctypes`` costs ~2.5 us a call, a sizeable part
        of a sampler round's host time."""
        if getattr(self, "_st", None) is None:
            k = min(self.max_draws, self._STAGE_DRAWS)
            bl, mv, out = np.empty((k, self.B)), np.empty((k, self.model_len)), np.empty((k, self.outlen))
            self._st = (bl, mv, out, bl.ctypes.data, mv.ctypes.data, out.ctypes.data)
        return self._st

    def submit_rows(self, blens, model_vecs):
        """Start an evaluation of n <= 128 draws (phy_eval_submit) and return
        at once; ``wait_rows`` collects its raw output rows."""
        blens, mv = np.asarray(blens, np.float64), np.asarray(model_vecs, np.float64)
        if blens.ndim == 1:
            blens, mv = blens[None], mv.reshape(1, -1)
        n = blens.shape[0]
        if blens.shape != (n, self.B) or mv.shape != (n, self.model_len):
            raise ValueError("bad shapes: blens %s model %s" % (blens.shape, mv.shape))
        sbl, smv, _, pbl, pmv, _ = self._stage()
        if n <= sbl.shape[0]:
            sbl[:n] = blens  # phy_eval_submit stages them into pinned memory before it returns
            smv[:n] = mv
        else:  # beyond the limit: phy_eval_submit reports it
            blens, mv = np.ascontiguousarray(blens), np.ascontiguousarray(mv)
            pbl, pmv = blens.ctypes.data, mv.ctypes.data
        _lib.check(self.lib.phy_eval_submit(self.ctx, n, pbl, pmv), "phy_eval_submit")
        self._pending = n

    def native_submit_wait(self, n):
        """(context, phy_eval_submit, phy_eval_wait addresses, row length)
        for a native caller that evaluates up to n draws per call through the
        submit / wait pair (nuts.py's native sampling loop), or None when n
        exceeds what one submit takes."""
        if n > min(self.max_draws, self._STAGE_DRAWS) or getattr(self, "ctx", None) is None:
            return None
        return (self.ctx.value, ctypes.cast(self.lib.phy_eval_submit, ctypes.c_void_p).value,
                ctypes.cast(self.lib.phy_eval_wait, ctypes.c_void_p).value, self.outlen)

    def wait_rows(self):
        """The rows [n, outlen] of the evaluation ``submit_rows`` started."""
        n, self._pending = self._pending, 0
        _, _, out, _, _, pout = self._stage()
        _lib.check(self.lib.phy_eval_wait(self.ctx, pout), "phy_eval_wait")
        return out[:n].copy()

    def evaluate(self, blens, model_vec, site_ll=False):
        return self.evaluate_batch(blens, model_vec, site_ll)[0]

    def evaluate_device(self, d_blens, d_model, d_out, d_site_ll=0, n_draws=1, stream=0):
        """Device-pointer path (ints), asynchronous on ``stream``."""
        _lib.check(self.lib.phy_eval_device(self.ctx, int(n_draws), ctypes.c_void_p(d_blens),
                                            ctypes.c_void_p(d_model), ctypes.c_void_p(d_out),
                                            ctypes.c_void_p(d_site_ll) if d_site_ll else None,
                                            ctypes.c_void_p(stream) if stream else None),
                   "phy_eval_device")

    def pruning_loglik(self, blens, model_vec):
        """``pruning_loglik(blens)`` of eigen/prune_stan.hpp:9-17: returns
        ``(log_P, grad)`` -- the value and the precomputed gradient."""
        blens = np.ascontiguousarray(blens, dtype=np.float64)
        mv = np.ascontiguousarray(model_vec, dtype=np.float64)
        grad = np.empty(self.B)
        val = self.lib.phy_pruning_loglik(self.ctx, _ptr(blens), _ptr(mv), _ptr(grad))
        if np.isnan(val):
            msg = self.lib.phy_last_error().decode(errors="replace")
            if msg:
                raise _lib.PhyloHipError("phy_pruning_loglik: " + msg)
        return val, grad

    def sync(self):
        _lib.check(self.lib.phy_sync(self.ctx), "phy_sync")

    def set_tuning(self, wg_budget=0, cols=0, lds_budget=0):
        """Persistent-workgroup budget, columns per lane (0 = automatic, 1, 2)
        and LDS bytes per workgroup (0 = keep); see include/phylo_hip_diag.h."""
        _lib.check(self.lib.phy_set_tuning(self.ctx, int(wg_budget), int(cols), int(lds_budget)),
                   "phy_set_tuning")

    def set_deep_stack(self, mode=0):
        """Deep-stack placement: 0 automatic, 1 LDS, 2 global (replans)."""
        _lib.check(self.lib.phy_set_deep_stack(self.ctx, int(mode)), "phy_set_deep_stack")

    def set_recompute(self, on=True):
        """Rebuild cherries in the reverse half instead of storing them (replans)."""
        _lib.check(self.lib.phy_set_recompute(self.ctx, int(bool(on))), "phy_set_recompute")

    def lds_plan(self):
        vals = [ctypes.c_int() for _ in range(3)]
        _lib.check(self.lib.phy_lds_plan(self.ctx, *[ctypes.byref(v) for v in vals]), "phy_lds_plan")
        out = dict(zip(("n_chunks", "matrices_per_chunk", "lds_bytes"), [v.value for v in vals]))
        out["cols"] = self.lib.phy_columns_per_lane(self.ctx)
        out["deep_lds_entries"] = self.lib.phy_deep_stack_in_lds(self.ctx)
        out["recomputed"] = self.lib.phy_recomputed_partials(self.ctx)
        return out

    def set_output(self, compact=False):
        """compact: output rows stop after the model-parameter gradients (no
        dL/dP block: 1 + B + 2C + 14 doubles per draw, what a sampler needs)."""
        _lib.check(self.lib.phy_set_output(self.ctx, int(bool(compact))), "phy_set_output")
        self.outlen = self.lib.phy_output_len(self.ctx)
        self._st = None  # the staging rows follow the row length

    def set_engine(self, mode=0):
        """0 automatic, 1 pattern sweep (its quad form for calls of <= 32
        draws), 2 class sweep (site repeats).  Round 3's resident class sweep
        (mode 3) is retired: phy_set_engine refuses it."""
        if isinstance(mode, str):
            mode = {"auto": 0, "pattern": 1, "class": 2}[mode]
        _lib.check(self.lib.phy_set_engine(self.ctx, int(mode)), "phy_set_engine")

    def prefer_latency_engine(self, probe=True, calls=24):
        """For host-driven samplers (a few draws per call, one call per
        leapfrog / ELBO round): the pattern sweep (its quad form for <= 32
        draws) -- faster than round 3's resident class sweep on every
        workload (fluA 99.8 against 132 us per 4-draw call) -- unless the
        automatic choice is the class sweep (a large alignment); then both are
        measured here (``calls`` synchronous calls of ``max_draws`` synthetic
        draws -- branch lengths 0.05, uniform frequencies, unit rates -- on
        each, in two alternating rounds, the lower median kept) and the
        faster is kept.  The choice affects speed only: both engines pass the
        same parity tests.  probe=False: the automatic engine's choice.
        Returns the name; timings (us per call), when measured, are in
        ``self.latency_probe``."""
        self.set_engine("auto")
        if self.engine() == "pattern" or not probe:
            return self.engine()
        import time
        n = self.max_draws
        bl = np.full((n, self.B), 0.05)
        mv = np.repeat(self.model_vector([0.25] * 4, [1.0] * 6, [1.0] * self.C, [1.0 / self.C] * self.C)[None], n,
                       axis=0)
        times = {"pattern": [], "class": []}
        for rnd in range(2):
            for name in ("pattern", "class"):
                self.set_engine(name)
                for _ in range(3):
                    self.evaluate_rows(bl, mv)
                for _ in range(calls // 2):
                    t0 = time.perf_counter()
                    self.evaluate_rows(bl, mv)
                    times[name].append(time.perf_counter() - t0)
        med = {k: 1e6 * float(np.median(v)) for k, v in times.items()}
        self.latency_probe = med
        self.set_engine(min(med, key=med.get))
        return self.engine()

    def engine(self):
        """The engine the next launch uses: "pattern" or "class"."""
        return ("pattern", "class")[self.lib.phy_engine(self.ctx)]

    def class_info(self):
        ll = [ctypes.c_longlong() for _ in range(3)]
        ii = [ctypes.c_int() for _ in range(4)]
        _lib.check(self.lib.phy_class_info(self.ctx, ctypes.byref(ll[0]), ctypes.byref(ii[0]), ctypes.byref(ii[1]),
                                           ctypes.byref(ll[1]), ctypes.byref(ll[2]), ctypes.byref(ii[2]),
                                           ctypes.byref(ii[3])), "phy_class_info")
        fl, nc, big = ctypes.c_int(), ctypes.c_int(), ctypes.c_longlong()
        _lib.check(self.lib.phy_class_clades(self.ctx, ctypes.byref(fl), ctypes.byref(nc), ctypes.byref(big)),
                   "phy_class_clades")
        cl, clo, ctop = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.phy_class_chain(self.ctx, ctypes.byref(cl), ctypes.byref(clo), ctypes.byref(ctop)),
                   "phy_class_chain")
        pr, cs, po = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.phy_class_fused(self.ctx, ctypes.byref(pr), ctypes.byref(cs), ctypes.byref(po)),
                   "phy_class_fused")
        return dict(classes=ll[0].value, levels=ii[0].value, root_classes=ii[1].value, stage=ll[1].value,
                    staged=ll[2].value, tiles=ii[2].value, spans=ii[3].value, clade_levels=fl.value,
                    clades=nc.value, clade_max=big.value, chain_levels=cl.value, chain_lowest=clo.value,
                    chain_top_classes=ctop.value, level_pairs=pr.value,
                    chunk_spans=cs.value, parent_order_levels=po.value)

    def quad_plan(self):
        """The small-call sweep's plan: waves per category, schedule length in
        program steps, LDS hand-off slots (include/phylo_hip_diag.h phy_quad_plan)."""
        w, sp, sl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.phy_quad_plan(self.ctx, ctypes.byref(w), ctypes.byref(sp), ctypes.byref(sl)),
                   "phy_quad_plan")
        return dict(waves=w.value, span=sp.value, slots=sl.value)

    def timing_start(self):
        _lib.check(self.lib.phy_timing_start(self.ctx), "phy_timing_start")

    def timing_read(self):
        ms = ctypes.c_double()
        n = ctypes.c_int()
        _lib.check(self.lib.phy_timing_read(self.ctx, ctypes.byref(ms), ctypes.byref(n)),
                   "phy_timing_read")
        return ms.value, n.value
