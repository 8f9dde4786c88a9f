"""Debug helper: one random case on the GPU vs the oracle, per output array."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests import cases
from phylostan_amd.engine import TreeLikelihood

seed, S, P, C, model, cols, wg, mode, lds = [int(x) if x.lstrip('-').isdigit() else x for x in sys.argv[1:10]]
case = cases.random_case(seed, S=S, P=P, C=C, model=model)
eng = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, max_draws=1)
eng.set_tuning(wg, cols, lds)
eng.set_deep_stack(mode)
print(eng.program_info(), eng.lds_plan())
res = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
ref = case.oracle()
for k in ("dLdP", "grad_blens", "grad_rs", "grad_ps", "grad_freq_root"):
    a, b = np.asarray(getattr(res, k)), np.asarray(ref[k])
    print(k, np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))
print("gpu", res.grad_freq_root, "\nref", ref["grad_freq_root"])
