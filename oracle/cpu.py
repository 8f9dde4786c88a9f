"""ctypes binding of oracle/liboracle_cpu.so -- TEST INFRASTRUCTURE ONLY."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def load():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle_cpu.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle_cpu.so not built: make -C oracle")
        lib = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        lib.oracle_eval.restype = ctypes.c_int
        lib.oracle_eval.argtypes = [ctypes.c_int] * 5 + [vp] * 7 + [ctypes.c_int]
        _LIB = lib
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def evaluate(tipcodes, weights, peel0, rooted, kind, model_vec, blens, C, site_ll=False, nthreads=1):
    """Output vector (include/phylo_hip.h layout) and optional per-site log L."""
    lib = load()
    tipcodes = np.ascontiguousarray(tipcodes, dtype=np.uint8)
    S, P = tipcodes.shape
    B = 2 * S - 2 if rooted else 2 * S - 3
    w = np.ascontiguousarray(weights, dtype=np.float64)
    peel = np.ascontiguousarray(peel0, dtype=np.int32)
    mv = np.ascontiguousarray(model_vec, dtype=np.float64)
    bl = np.ascontiguousarray(blens, dtype=np.float64)
    og = 1 + B + 2 * C + 4 + 10
    out = np.empty(og + 16 * C * B)
    sl = np.empty(P) if site_ll else None
    lib.oracle_eval(S, P, C, int(rooted), int(kind), _p(tipcodes), _p(w), _p(peel), _p(mv), _p(bl),
                    _p(out), _p(sl), int(nthreads))
    if int(kind) != 0:  # HKY / GTR: exchangeability and frequency gradients by the host chain rule
        from phylostan_amd import models
        gr, gf = models.q_param_gradients(out[og:].reshape(C, B, 4, 4), bl, mv[10:10 + C], mv[:4], mv[4:10],
                                          out[1 + B + 2 * C:1 + B + 2 * C + 4])
        out[og - 10:og - 4] = gr
        out[og - 4:og] = gf
    return out, sl
