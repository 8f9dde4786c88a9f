"""GPU: a tree whose C * B needs more than 64 KiB of epilogue LDS (ADVICE r03:
finalize_kernel's LDS is (C*B + 16 + 1024 + QG_SHARED) doubles, opted in to
the 160 KiB cap at phy_create) -- 430 taxa (B = 858), C = 16: C * B =
13,728, 121 KB of finalize LDS (more taxa underflow the per-site likelihood
without rescaling, as in the reference) -- on the column sweep's finalize
(1, 4 and 32 draws: its records do not fit the quad sweep's LDS plan) and the
class sweep's epilogue.  Every gradient
against the oracle at the parity bar (tests/test_gpu_parity.py)."""
import numpy as np
import pytest
import torch  # noqa: F401 -- torch's own HIP runtime must load before the engine's

from tests import cases
from tests.test_gpu_parity import RTOL_G, RTOL_LL, _close, check_case

pytestmark = pytest.mark.gpu


def _case():
    return cases.random_case(901, S=430, P=300, C=16, model="GTR")


def _engine(case, max_draws, engine="auto"):
    from phylostan_amd.engine import TreeLikelihood
    eng = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C,
                         max_draws=max_draws)
    eng.set_engine(engine)
    return eng


@pytest.mark.parametrize("engine", ["pattern", "class"])
def test_large_cb_single_eval_vs_oracle(engine):
    case = _case()
    assert case.C * (2 * 430 - 2) > 6800
    check_case(case, _engine(case, 1, engine))


@pytest.mark.parametrize("n", [4, 32])
def test_large_cb_batched_rows_vs_oracle(n):
    """The sampler's and a batch's shapes through finalize_kernel (121 KB of
    LDS)."""
    case = _case()
    eng = _engine(case, n, "pattern")
    rng = np.random.default_rng(5)
    bl = case.blens[None, :] * rng.uniform(0.8, 1.25, (n, case.blens.size))
    mv = np.repeat(case.model_vec()[None], n, axis=0)
    rows = eng.evaluate_rows(bl, mv)
    for k in (0, n - 1):
        c = cases.Case(case.name, case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, bl[k],
                       case.freqs, case.rates, case.rs, case.ps)
        ref = c.oracle()
        assert abs(rows[k, 0] - ref["loglik"]) <= RTOL_LL * abs(ref["loglik"])
        _close(rows[k, 1:1 + eng.B], ref["grad_blens"], RTOL_G, "grad_blens draw %d" % k)
