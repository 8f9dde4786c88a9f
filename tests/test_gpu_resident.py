"""GPU parity of the resident class sweep (the class sweep with each
(draw, category)'s whole state in LDS, csrc/resident_engine.inc) against the
CPU oracle, through the C-ABI with phy_set_engine(3).

Same bar as tests/test_gpu_parity.py: per-site and total log L rel 1e-10,
every gradient rel 1e-9 of its array's largest entry.
"""
import numpy as np
import pytest

from phylostan_amd import _lib
from tests import cases
from tests.test_gpu_parity import RTOL_G, RTOL_LL, _close, _engine, check_case

pytestmark = pytest.mark.gpu


def _res_engine(case, max_draws=1):
    eng = _engine(case, max_draws=max_draws)
    eng.set_engine("resident")
    assert eng.engine() == "resident"
    return eng


@pytest.mark.parametrize("make", [cases.fluA_case, cases.hcv_case], ids=["fluA_HKY_W4", "HCV_GTR_W4"])
def test_resident_config_datasets(make):
    case = make()
    check_case(case, _res_engine(case))


@pytest.mark.parametrize("seed,S,P,C,model,cat", [
    (1, 3, 1, 1, "JC69", False),      # smallest tree, single pattern
    (2, 5, 1, 1, "JC69", False),
    (3, 12, 63, 3, "GTR", False),
    (4, 12, 130, 4, "HKY", False),
    (5, 40, 90, 2, "GTR", True),      # caterpillar: one node per level
    (6, 9, 100, 8, "HKY", False),     # many categories
    (7, 30, 130, 4, "GTR", False),    # chunks of 64+ classes per node, long segments
    (8, 60, 30, 1, "GTR", False),     # many levels, one category
])
def test_resident_random_trees(seed, S, P, C, model, cat):
    case = cases.random_case(seed, S=S, P=P, C=C, model=model, rooted=True, caterpillar=cat)
    check_case(case, _res_engine(case))


def test_resident_all_masks_and_ambiguous_tips():
    """Every 4-bit tip mask (extra matrix records) and all-ambiguous tips."""
    base = cases.random_case(40, S=16, P=150, C=4, model="GTR")
    rng = np.random.default_rng(40)
    codes = rng.integers(1, 16, size=(16, 150)).astype(np.uint8)
    codes[3, :] = 15
    case = cases.Case("masks", codes, base.weights, base.peel0, True, "GTR", 4, base.blens, base.freqs,
                      base.rates, base.rs, base.ps)
    check_case(case, _res_engine(case))


def test_resident_duplicate_columns_share_a_root_class():
    base = cases.random_case(71, S=10, P=80, C=2, model="HKY")
    codes = np.concatenate([base.tipcodes, base.tipcodes[:, :20]], axis=1)
    w = np.concatenate([base.weights, np.arange(1, 21, dtype=np.float64)])
    case = cases.Case("dup", codes, w, base.peel0, True, "HKY", 2, base.blens, base.freqs, base.rates,
                      base.rs, base.ps)
    check_case(case, _res_engine(case))


def test_resident_batched_draws_match_single():
    base = cases.fluA_case()
    rng = np.random.default_rng(3)
    n = 7
    eng = _res_engine(base, max_draws=n)
    blens = base.blens[None, :] * rng.uniform(0.5, 1.5, (n, 1))
    mvs = np.stack([cases.models.model_vector(rng.dirichlet([20] * 4), base.rates, base.rs,
                                              base.ps) for _ in range(n)])
    res = eng.evaluate_batch(blens, mvs, site_ll=True)
    for k in range(n):
        c = cases.Case("d%d" % k, base.tipcodes, base.weights, base.peel0, True, base.model, base.C, blens[k],
                       mvs[k][:4], base.rates, base.rs, base.ps)
        check_case(c, eng, res[k])


def test_resident_deterministic_and_agrees_with_pattern_sweep():
    case = cases.hcv_case()
    eng = _res_engine(case, max_draws=2)
    a = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    b = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    assert a.loglik == b.loglik
    assert np.array_equal(a.dLdP, b.dLdP) and np.array_equal(a.site_ll, b.site_ll)
    eng.set_engine("pattern")
    c = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    np.testing.assert_allclose(a.site_ll, c.site_ll, rtol=RTOL_LL, atol=1e-12)
    _close(a.dLdP, c.dLdP, RTOL_G, "dLdP")
    _close(a.grad_rates, c.grad_rates, 1e-8, "grad_rates")


def test_resident_zero_likelihood_is_minus_inf():
    """ps = 0 -> L = 0 -> log L = -inf (the sampler rejects the draw)."""
    case = cases.hcv_case()
    eng = _res_engine(case)
    mv = case.model_vec().copy()
    mv[10 + case.C:] = 0.0
    res = eng.evaluate(case.blens, mv, site_ll=True)
    assert res.loglik == -np.inf


def test_resident_refuses_state_beyond_lds():
    """~7,600 distinct subtree classes (243 KB per draw-category) do not fit."""
    case = cases.random_case(5, S=40, P=200, C=2, model="GTR", rooted=True, caterpillar=True)
    eng = _engine(case)
    with pytest.raises(_lib.PhyloHipError):
        eng.set_engine("resident")
    assert eng.resident_info()["lds_bytes"] == 0


def test_resident_refuses_unrooted():
    case = cases.ds1_case()
    eng = _engine(case)
    with pytest.raises(_lib.PhyloHipError):
        eng.set_engine("resident")


@pytest.mark.parametrize("block", range(4))
def test_resident_fuzz_small_rooted(block):
    """24 random rooted trees (3..48 taxa, 1..160 patterns, C 1..6, JC69 /
    HKY / GTR, 10-40 % ambiguous tips, some caterpillars) against the oracle."""
    rng = np.random.default_rng(500 + block)
    for k in range(6):
        S = int(rng.integers(3, 49))
        P = int(rng.integers(1, 161))
        C = int(rng.integers(1, 7))
        model = ("JC69", "HKY", "GTR")[int(rng.integers(0, 3))]
        case = cases.random_case(1000 * block + k, S=S, P=P, C=C, model=model, rooted=True,
                                 caterpillar=bool(rng.random() < 0.3), ambiguous=float(rng.uniform(0.1, 0.4)))
        eng = _engine(case)
        try:
            eng.set_engine("resident")
        except _lib.PhyloHipError:  # class state beyond LDS: the refusal is the contract
            assert eng.resident_info()["lds_bytes"] == 0
            continue
        check_case(case, eng)
