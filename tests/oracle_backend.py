"""A CPU stand-in for ``TreeLikelihood`` built on the numpy oracle.

TEST INFRASTRUCTURE ONLY: it lets the host-side posterior, samplers and CLI
be exercised on the CPU container (no GPU) against the oracle.  The product
path never imports it; on the GPU box the same tests use the HIP engine.
"""
from types import SimpleNamespace

import numpy as np

from oracle import numpy_pruner as npr
from phylostan_amd import models


class OracleLikelihood:
    def __init__(self, tipcodes, weights, peel0, rooted, model, C, **_):
        self.tipcodes = np.asarray(tipcodes, np.uint8)
        self.weights = np.asarray(weights, np.float64)
        self.peel0 = np.asarray(peel0, np.int64)
        self.rooted = bool(rooted)
        self.kind = npr.MODEL_IDS[model] if isinstance(model, str) else int(model)
        self.C = int(C)
        self.S, self.P = self.tipcodes.shape
        self.B = 2 * self.S - 2 if rooted else 2 * self.S - 3
        self.calls = 0

    def evaluate_batch(self, blens, model_vecs, site_ll=False):
        blens = np.atleast_2d(np.asarray(blens, np.float64))
        mvs = np.atleast_2d(np.asarray(model_vecs, np.float64))
        C = self.C
        out = []
        for b, mv in zip(blens, mvs):
            self.calls += 1
            freqs, rates, rs, ps = mv[:4], mv[4:10], mv[10:10 + C], mv[10 + C:10 + 2 * C]
            q = rates if self.kind == npr.GTR else rates
            P, Q = npr.model_matrices(self.kind, freqs, q, b, rs)
            fr = freqs if self.kind != npr.JC69 else np.full(4, 0.25)
            r = npr.prune(self.tipcodes, self.weights, self.peel0, self.rooted, P, fr, ps, Q=Q, blens=b, rs=rs)
            if self.kind == npr.JC69:
                gr, gf = np.zeros(6), np.zeros(4)
            else:  # the host chain rule (the engine does it on the device)
                gr, gf = models.q_param_gradients(r["dLdP"], b, rs, freqs, rates, r["grad_freq_root"])
            out.append(SimpleNamespace(loglik=float(r["loglik"]), grad_blens=r["grad_blens"], grad_rs=r["grad_rs"],
                                       grad_ps=r["grad_ps"], grad_freq_root=r["grad_freq_root"], dLdP=r["dLdP"],
                                       grad_rates=gr, grad_freqs=gf, site_ll=r["site_ll"] if site_ll else None))
        return out

    def evaluate(self, blens, model_vec, site_ll=False):
        return self.evaluate_batch(blens, model_vec, site_ll)[0]

    def close(self):
        pass
