"""Diagnostic: per-phase cycle split of the sweep kernel (stamp build)."""
import ctypes, os, sys
import numpy as np
os.environ["PHYLO_HIP_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "phylostan_amd", "libphylo_hip_stamp.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from phylostan_amd.engine import TreeLikelihood
from phylostan_amd import _lib
from tests import cases
lib = _lib.load()
lib.phy_debug_stamps.restype = ctypes.c_int
lib.phy_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
for draws in (1, 512):
    c = cases.fluA_case()
    eng = TreeLikelihood(c.tipcodes, c.weights, c.peel0, True, "HKY", 4, max_draws=draws)
    bl = np.tile(c.blens, (draws, 1)); mv = np.tile(c.model_vec(), (draws, 1))
    for _ in range(3): eng.evaluate_batch(bl, mv)
    buf = np.zeros(eng.lib.phy_output_len(eng.ctx) and 1 << 20, dtype=np.uint64)
    n = lib.phy_debug_stamps(eng.ctx, buf.ctypes.data_as(ctypes.c_void_p), buf.size)
    gx = min(4, max(1, (512 + draws - 1) // draws))
    st = buf[: gx * draws * 4 * 8].reshape(-1, 8).astype(np.int64)
    d = np.diff(st[:, :6], axis=1)
    clk = (st[:, 5] - st[:, 0]) / np.maximum(st[:, 7] - st[:, 6], 1) * 100.0  # MHz
    print("draws", draws, "waves", st.shape[0], "median cycles: start->fwd %d fwd %d root %d rev %d end %d" % tuple(np.median(d, 0)),
          "clock MHz median %.0f" % np.median(clk))
