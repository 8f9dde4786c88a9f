"""GPU parity of the class sweep (site repeats, SURVEY.md 8a row a10 --
the exact form of the reference's column-reuse cache, pruner/tree.cpp:140-174)
against the CPU oracle, through the C-ABI with phy_set_engine(2).

Same bar as tests/test_gpu_parity.py: per-site and total log L rel 1e-10,
every gradient rel 1e-9 of its array's largest entry.
"""
import os

import numpy as np
import pytest

from tests import cases
from tests.test_gpu_parity import RTOL_G, RTOL_LL, _close, _engine, check_case

pytestmark = pytest.mark.gpu


def _class_engine(case, max_draws=1):
    eng = _engine(case, max_draws=max_draws)
    eng.set_engine("class")
    assert eng.engine() == "class"
    return eng


@pytest.mark.parametrize("make", [cases.fluA_case, cases.hcv_case, cases.ds1_case],
                         ids=["fluA_HKY_W4", "HCV_GTR_W4", "DS1_JC69_unrooted"])
def test_class_sweep_config_datasets(make):
    case = make()
    eng = _class_engine(case)
    info = eng.class_info()
    assert 0 < info["classes"] < (case.S - 2) * case.P
    check_case(case, eng)


@pytest.mark.parametrize("seed,S,P,C,model,rooted,cat", [
    (1, 5, 1, 1, "JC69", True, False),       # single pattern
    (2, 12, 63, 3, "GTR", True, False),
    (3, 12, 130, 4, "HKY", True, False),
    (4, 17, 257, 5, "GTR", False, False),    # unrooted
    (5, 40, 200, 2, "GTR", True, True),      # caterpillar
    (6, 40, 200, 4, "JC69", False, True),    # unrooted caterpillar
    (7, 128, 3000, 4, "GTR", True, False),   # long segments, many tiles
    (8, 9, 100, 8, "HKY", True, False),
    (9, 300, 500, 4, "GTR", True, False),    # many levels
])
def test_class_sweep_random_trees(seed, S, P, C, model, rooted, cat):
    case = cases.random_case(seed, S=S, P=P, C=C, model=model, rooted=rooted, caterpillar=cat)
    check_case(case, _class_engine(case))


def test_class_sweep_repetitive_alignment():
    """Few distinct states per column (most subtrees repeat): long
    aggregation segments crossing many 64-position tiles."""
    rng = np.random.default_rng(70)
    base = cases.random_case(70, S=48, P=5000, C=4, model="GTR")
    codes = np.where(rng.random((48, 5000)) < 0.9, 1, rng.choice([1, 2, 4, 8, 15], size=(48, 5000)))
    codes = codes.astype(np.uint8)
    case = cases.Case("rep", codes, base.weights, base.peel0, True, "GTR", 4, base.blens, base.freqs,
                      base.rates, base.rs, base.ps)
    eng = _class_engine(case)
    assert eng.class_info()["spans"] > 0
    check_case(case, eng)


def test_class_sweep_duplicate_columns_share_a_root_class():
    """Patterns that differ only in raw symbols map to the same tip codes
    (e.g. N and -): they share a root class whose weight is the sum; every
    pattern still gets its own site log-likelihood."""
    base = cases.random_case(71, S=10, P=80, C=2, model="HKY")
    codes = np.concatenate([base.tipcodes, base.tipcodes[:, :20]], axis=1)
    w = np.concatenate([base.weights, np.arange(1, 21, dtype=np.float64)])
    case = cases.Case("dup", codes, w, base.peel0, True, "HKY", 2, base.blens, base.freqs, base.rates,
                      base.rs, base.ps)
    eng = _class_engine(case)
    assert eng.class_info()["root_classes"] == 80
    check_case(case, eng)


def test_class_sweep_batched_draws_match_single():
    base = cases.hcv_case()
    rng = np.random.default_rng(3)
    n = 5
    eng = _class_engine(base, max_draws=n)
    blens = base.blens[None, :] * rng.uniform(0.5, 1.5, (n, 1))
    mvs = np.stack([cases.models.model_vector(base.freqs, base.rates * rng.uniform(0.8, 1.2, 6), base.rs,
                                              base.ps) for _ in range(n)])
    res = eng.evaluate_batch(blens, mvs, site_ll=True)
    for k in range(n):
        c = cases.Case("d%d" % k, base.tipcodes, base.weights, base.peel0, True, "GTR", 4, blens[k], base.freqs,
                       mvs[k][4:10], base.rs, base.ps)
        check_case(c, eng, res[k])


def test_class_sweep_deterministic_and_agrees_with_pattern_sweep():
    case = cases.random_case(72, S=64, P=2000, C=4, model="GTR")
    eng = _class_engine(case)
    a = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    b = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    assert a.loglik == b.loglik
    assert np.array_equal(a.dLdP, b.dLdP) and np.array_equal(a.site_ll, b.site_ll)
    eng.set_engine("pattern")
    assert eng.engine() == "pattern"
    c = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    np.testing.assert_allclose(a.site_ll, c.site_ll, rtol=RTOL_LL, atol=1e-12)
    _close(a.dLdP, c.dLdP, RTOL_G, "dLdP")


def _with_clade(case, value, max_draws=1):
    # (chain-free plans: the top chain starts above the clade levels, so its
    # extent -- and the order of its dL/dP sums -- would follow the clade depth)
    old = os.environ.get("PHY_CLADE"), os.environ.get("PHY_CHAIN")
    if value is None:
        os.environ.pop("PHY_CLADE", None)
    else:
        os.environ["PHY_CLADE"] = str(value)
    os.environ["PHY_CHAIN"] = "0"
    try:
        return _class_engine(case, max_draws=max_draws)
    finally:
        for k, v in zip(("PHY_CLADE", "PHY_CHAIN"), old):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("seed,S,P,C,model,rooted,cat", [
    (7, 128, 3000, 4, "GTR", True, False),
    (9, 300, 500, 4, "GTR", True, False),
    (4, 17, 257, 5, "GTR", False, False),
    (5, 40, 200, 2, "GTR", True, True),
])
def test_class_clades_bitwise_equal_to_level_launches(seed, S, P, C, model, rooted, cat):
    """Bottom clades (levels 1..Lc fused, one workgroup per clade) run the
    same chunks / tiles / spans in the same order as the per-level launches:
    outputs bitwise equal for the automatic plan and forced depths, and the
    forced-deepest plan still matches the oracle."""
    case = cases.random_case(seed, S=S, P=P, C=C, model=model, rooted=rooted, caterpillar=cat)
    ref_eng = _with_clade(case, 0)
    assert ref_eng.class_info()["clade_levels"] == 0
    ref = ref_eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    levels = ref_eng.class_info()["levels"]
    for value in (None, 1, 3, levels):
        eng = _with_clade(case, value)
        info = eng.class_info()
        if value is not None:
            assert info["clade_levels"] == max(0, min(value, levels - 2))
        got = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
        assert got.loglik == ref.loglik
        assert np.array_equal(got.site_ll, ref.site_ll)
        assert np.array_equal(got.dLdP, ref.dLdP) and np.array_equal(got.grad_blens, ref.grad_blens)
        assert np.array_equal(got.grad_rates, ref.grad_rates) and np.array_equal(got.grad_freqs, ref.grad_freqs)
    check_case(case, _with_clade(case, levels))


def test_class_clades_repetitive_alignment_bitwise():
    """Long tile-crossing segments inside the fused levels (FIX phases inside
    the clade workgroups)."""
    rng = np.random.default_rng(70)
    base = cases.random_case(70, S=48, P=5000, C=4, model="GTR")
    codes = np.where(rng.random((48, 5000)) < 0.9, 1, rng.choice([1, 2, 4, 8, 15], size=(48, 5000)))
    case = cases.Case("rep", codes.astype(np.uint8), base.weights, base.peel0, True, "GTR", 4, base.blens,
                      base.freqs, base.rates, base.rs, base.ps)
    ref = _with_clade(case, 0).evaluate(case.blens, case.model_vec(), site_ll=True)
    eng = _with_clade(case, 50)
    assert eng.class_info()["clade_levels"] > 0
    got = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    assert got.loglik == ref.loglik and np.array_equal(got.dLdP, ref.dLdP) and np.array_equal(got.site_ll, ref.site_ll)


def _assert_rows_equal(a, b):
    assert a.loglik == b.loglik
    assert np.array_equal(a.site_ll, b.site_ll)
    for k in ("dLdP", "grad_blens", "grad_rs", "grad_ps", "grad_freq_root", "grad_rates", "grad_freqs"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k


def test_class_epilogue_stress_bitwise_over_many_calls():
    """The class epilogue's cross-workgroup hand-offs (write-through stores,
    a per-draw ticket, the last workgroup's acquire) under repetition: 10,000
    back-to-back device-path evaluations of a 200-taxon alignment in one
    process, every output row bitwise equal to the first (a stale read
    anywhere would show as a differing row)."""
    import torch
    case = cases.random_case(91, S=200, P=4000, C=4, model="GTR")
    eng = _class_engine(case, max_draws=2)
    dev = torch.device("cuda:0")
    bl = torch.tensor(np.stack([case.blens, case.blens * 1.1]), device=dev)
    mv = torch.tensor(np.stack([case.model_vec()] * 2), device=dev)
    out = torch.zeros((2, eng.outlen), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    stream = torch.cuda.Stream(dev)  # the engine's launches and torch's compares in one order
    st = stream.cuda_stream
    with torch.cuda.stream(stream):
        eng.evaluate_device(bl.data_ptr(), mv.data_ptr(), out.data_ptr(), n_draws=2, stream=st)
        first = out.clone()
        stream.synchronize()
        assert np.isfinite(first.cpu().numpy()).all() and first[0, 0].item() < 0.0
        bad = torch.zeros((), dtype=torch.int64, device=dev)
        for _ in range(10000):
            eng.evaluate_device(bl.data_ptr(), mv.data_ptr(), out.data_ptr(), n_draws=2, stream=st)
            bad += (out != first).any().to(torch.int64)
        stream.synchronize()
    assert int(bad.item()) == 0


def _chain_pair(case, monkeypatch, max_draws=1):
    """The same plan with and without the top chain (PHY_CHAIN=0)."""
    monkeypatch.setenv("PHY_CHAIN", "0")
    plain = _class_engine(case, max_draws=max_draws)
    monkeypatch.delenv("PHY_CHAIN")
    chained = _class_engine(case, max_draws=max_draws)
    assert plain.class_info()["chain_levels"] == 0
    return chained, plain


@pytest.mark.parametrize("make", [cases.fluA_case, cases.hcv_case, cases.ds1_case, "syn200k", "caterpillar",
                                  "caterpillar_c5"],
                         ids=["fluA", "HCV", "DS1_unrooted", "synthetic200k", "caterpillar_random",
                              "caterpillar_C5_chain_launch"])
def test_class_chain_equals_level_launches(make, monkeypatch):
    """The top chain (the single-node levels below the root in one forward and
    one reverse launch, one lane per top class) forms the level launches'
    forward values bit for bit -- site log-likelihoods and log-likelihood
    identical -- and the same gradients up to the order of the dL/dP sums of
    the chained branches (over top classes instead of each node's classes);
    both at the parity bar against the oracle."""
    if make == "syn200k":
        from phylostan_amd import synthetic
        pd, prm = synthetic.simulate(n_sites=200_000)
        case = cases.Case("syn200k", pd.tipcodes, pd.weights, pd.peel0, True, "GTR", 4, prm["blens"], prm["freqs"],
                          prm["rates"], prm["rs"], prm["ps"])
    elif make == "caterpillar":
        case = cases.random_case(5, S=40, P=2000, C=3, model="GTR", rooted=True, caterpillar=True)
    elif make == "caterpillar_c5":  # C > 4: the chain's own forward launch (the root recompute is C <= 4)
        case = cases.random_case(6, S=40, P=2000, C=5, model="GTR", rooted=True, caterpillar=True)
    else:
        case = make()
    chained, plain = _chain_pair(case, monkeypatch)
    info = chained.class_info()
    assert info["chain_levels"] >= 2, info
    a = chained.evaluate(case.blens, case.model_vec(), site_ll=True)
    b = plain.evaluate(case.blens, case.model_vec(), site_ll=True)
    assert a.loglik == b.loglik
    assert np.array_equal(a.site_ll, b.site_ll)
    for k in ("dLdP", "grad_blens", "grad_rs", "grad_ps", "grad_freq_root", "grad_rates", "grad_freqs"):
        x, y = np.asarray(getattr(a, k)), np.asarray(getattr(b, k))
        scale = max(float(np.max(np.abs(y))), 1e-300)
        assert float(np.max(np.abs(x - y))) <= 1e-12 * scale, k
    check_case(case, chained, a)


def test_class_chain_batched_draws_and_repeats(monkeypatch):
    """Chained plan, 16 draws per launch: every row equals its single-draw
    evaluation bit for bit, and repeated launches are bitwise reproducible."""
    case = cases.hcv_case()
    eng = _class_engine(case, max_draws=16)
    assert eng.class_info()["chain_levels"] >= 2
    rng = np.random.default_rng(3)
    bl = case.blens[None, :] * rng.uniform(0.7, 1.3, (16, case.blens.size))
    mv = np.repeat(case.model_vec()[None], 16, axis=0)
    rows = eng.evaluate_rows(bl, mv)
    assert np.array_equal(rows, eng.evaluate_rows(bl, mv))
    one = _class_engine(case, max_draws=1)
    for k in (0, 7, 15):
        assert np.array_equal(one.evaluate_rows(bl[k:k + 1], mv[k:k + 1])[0], rows[k])


def _pair_engines(case, monkeypatch, max_draws=1, pmax=None):
    """The same plan with forward level pairs (PHY_PAIR_MAX=pmax, or the
    default) and without (PHY_PAIR=0)."""
    monkeypatch.setenv("PHY_PAIR", "0")
    plain = _class_engine(case, max_draws=max_draws)
    monkeypatch.delenv("PHY_PAIR")
    if pmax is not None:
        monkeypatch.setenv("PHY_PAIR_MAX", str(pmax))
    paired = _class_engine(case, max_draws=max_draws)
    monkeypatch.delenv("PHY_PAIR_MAX", raising=False)
    assert plain.class_info()["level_pairs"] == 0
    return paired, plain


@pytest.mark.parametrize("make", [cases.fluA_case, cases.hcv_case, cases.ds1_case, "syn200k", "caterpillar", "deep"],
                         ids=["fluA", "HCV", "DS1_unrooted", "synthetic200k", "caterpillar_random", "random300"])
@pytest.mark.parametrize("pmax", [None, 1 << 40], ids=["default", "all"])
def test_class_level_pairs_bitwise_equal_to_level_launches(make, pmax, monkeypatch):
    """Forward level pairs (cls_fwd2_kernel: two levels in one launch, the
    upper level recomputing its lower-level children from their children with
    the lower level's own arithmetic) leave every output bitwise equal to the
    per-level launches; at the parity bar against the oracle."""
    if make == "syn200k":
        from phylostan_amd import synthetic
        pd, prm = synthetic.simulate(n_sites=200_000)
        case = cases.Case("syn200k", pd.tipcodes, pd.weights, pd.peel0, True, "GTR", 4, prm["blens"], prm["freqs"],
                          prm["rates"], prm["rs"], prm["ps"])
    elif make == "caterpillar":
        case = cases.random_case(5, S=40, P=2000, C=3, model="GTR", rooted=True, caterpillar=True)
    elif make == "deep":
        case = cases.random_case(9, S=300, P=500, C=4, model="GTR", rooted=True)
    else:
        case = make()
    if pmax is not None:  # every level launched on its own (no clade, no chain), all of them paired
        monkeypatch.setenv("PHY_CLADE", "0")
        monkeypatch.setenv("PHY_CHAIN", "0")
    paired, plain = _pair_engines(case, monkeypatch, pmax=pmax)
    if pmax is not None:
        info = paired.class_info()
        assert info["level_pairs"] == (info["levels"] - 1) // 2, info
    a = paired.evaluate(case.blens, case.model_vec(), site_ll=True)
    b = plain.evaluate(case.blens, case.model_vec(), site_ll=True)
    _assert_rows_equal(a, b)
    check_case(case, paired, a)


def test_class_level_pairs_batched_draws_and_repeats(monkeypatch):
    """Paired plan, 8 draws per launch: rows bitwise equal to the unpaired
    plan's, and repeated launches bitwise reproducible."""
    case = cases.random_case(9, S=300, P=500, C=4, model="GTR", rooted=True)
    monkeypatch.setenv("PHY_CLADE", "0")
    paired, plain = _pair_engines(case, monkeypatch, max_draws=8, pmax=1 << 40)
    assert paired.class_info()["level_pairs"] >= 2
    rng = np.random.default_rng(5)
    bl = case.blens[None, :] * rng.uniform(0.7, 1.3, (8, case.blens.size))
    mv = np.repeat(case.model_vec()[None], 8, axis=0)
    rows = paired.evaluate_rows(bl, mv)
    assert np.array_equal(rows, plain.evaluate_rows(bl, mv))
    assert np.array_equal(rows, paired.evaluate_rows(bl, mv))


def _repetitive_case(seed=70, S=48, P=5000):
    """A repetitive alignment: long tile-crossing segments (one class of a
    small node collecting most of its parent's classes)."""
    rng = np.random.default_rng(seed)
    base = cases.random_case(seed, S=S, P=P, C=4, model="GTR")
    codes = np.where(rng.random((S, P)) < 0.9, 1, rng.choice([1, 2, 4, 8, 15], size=(S, P)))
    return cases.Case("rep", codes.astype(np.uint8), base.weights, base.peel0, True, "GTR", 4, base.blens,
                      base.freqs, base.rates, base.rs, base.ps)


@pytest.mark.parametrize("make", ["rep", "rep_noclade", "rep_nochain", cases.fluA_case, "syn200k"],
                         ids=["repetitive", "repetitive_no_clades", "repetitive_no_chain", "fluA", "synthetic200k"])
def test_class_revfix_bitwise_equal_to_fix_launches(make, monkeypatch):
    """Long tile-crossing segments summed by their REV chunk's wave
    (cls_rev_ls_kernel, fix_span's arithmetic) instead of a FIX launch per
    level: every output bitwise equal, batched draws too."""
    if make == "syn200k":
        from phylostan_amd import synthetic
        pd, prm = synthetic.simulate(n_sites=200_000)
        case = cases.Case("syn200k", pd.tipcodes, pd.weights, pd.peel0, True, "GTR", 4, prm["blens"], prm["freqs"],
                          prm["rates"], prm["rs"], prm["ps"])
    elif isinstance(make, str):
        case = _repetitive_case()
        if make == "rep_noclade":
            monkeypatch.setenv("PHY_CLADE", "0")
        if make == "rep_nochain":
            monkeypatch.setenv("PHY_CLADE", "0")
            monkeypatch.setenv("PHY_CHAIN", "0")
    else:
        case = make()
    monkeypatch.setenv("PHY_REVFIX", "0")
    plain = _class_engine(case, max_draws=3)
    monkeypatch.delenv("PHY_REVFIX")
    fused = _class_engine(case, max_draws=3)
    if isinstance(make, str) and make.startswith("rep_no"):
        assert fused.class_info()["chunk_spans"] > 0, fused.class_info()
    assert plain.class_info()["chunk_spans"] == 0
    a = fused.evaluate(case.blens, case.model_vec(), site_ll=True)
    b = plain.evaluate(case.blens, case.model_vec(), site_ll=True)
    _assert_rows_equal(a, b)
    check_case(case, fused, a)
    rng = np.random.default_rng(8)
    bl = case.blens[None, :] * rng.uniform(0.8, 1.2, (3, case.blens.size))
    mv = np.repeat(case.model_vec()[None], 3, axis=0)
    assert np.array_equal(fused.evaluate_rows(bl, mv), plain.evaluate_rows(bl, mv))


@pytest.mark.parametrize("make", [cases.fluA_case, cases.hcv_case, "syn200k"], ids=["fluA", "HCV", "synthetic200k"])
def test_class_root_chain_bitwise_equal_to_chain_forward_launch(make, monkeypatch):
    """The root recomputing the chain's top from the chain tables (no chain
    forward launch) gives every output bitwise equal to the plan that stores
    the chain's A in its own launch (PHY_ROOT_CHAIN=0), batched draws too."""
    if make == "syn200k":
        from phylostan_amd import synthetic
        pd, prm = synthetic.simulate(n_sites=200_000)
        case = cases.Case("syn200k", pd.tipcodes, pd.weights, pd.peel0, True, "GTR", 4, prm["blens"], prm["freqs"],
                          prm["rates"], prm["rs"], prm["ps"])
    else:
        case = make()
    monkeypatch.setenv("PHY_ROOT_CHAIN", "0")
    plain = _class_engine(case, max_draws=3)
    monkeypatch.delenv("PHY_ROOT_CHAIN")
    fused = _class_engine(case, max_draws=3)
    assert fused.class_info()["chain_levels"] >= 2
    a = fused.evaluate(case.blens, case.model_vec(), site_ll=True)
    b = plain.evaluate(case.blens, case.model_vec(), site_ll=True)
    _assert_rows_equal(a, b)
    rng = np.random.default_rng(12)
    bl = case.blens[None, :] * rng.uniform(0.8, 1.2, (3, case.blens.size))
    mv = np.repeat(case.model_vec()[None], 3, axis=0)
    assert np.array_equal(fused.evaluate_rows(bl, mv), plain.evaluate_rows(bl, mv))


@pytest.mark.parametrize("make", [cases.fluA_case, cases.hcv_case, "rep", "rep_nochain", "deep", "syn200k"],
                         ids=["fluA_no_chain", "HCV_chain", "repetitive", "repetitive_no_chain", "random300",
                              "synthetic200k"])
def test_class_parent_order_staging_bitwise_equal(make, monkeypatch):
    """Secondary-child staging written in the parent's class order and
    gathered by the RED tiles through the staging permutation (every level
    above the clades: PHY_STAGE_ORDER=0) against every contribution stored at
    its reduction position (PHY_STAGE_ORDER above any level's staging): the
    same values reduced in the same order -- every output bitwise equal,
    batched draws too, and at the parity bar against the oracle.  Covers the
    chain externals of a parent-order level (written by the chain reverse at
    their reduction positions: the permutation's identity entries)."""
    if make == "syn200k":  # (the automatic plan: clades, pairs, no chain)
        from phylostan_amd import synthetic
        pd, prm = synthetic.simulate(n_sites=200_000)
        case = cases.Case("syn200k", pd.tipcodes, pd.weights, pd.peel0, True, "GTR", 4, prm["blens"], prm["freqs"],
                          prm["rates"], prm["rs"], prm["ps"])
    else:
        # the small plans' levels above the bottom clades are mostly chain: no clades here, so the
        # levels below the chain launch on their own (with secondary children and chain externals)
        monkeypatch.setenv("PHY_CLADE", "0")
        if make in ("rep", "rep_nochain"):
            case = _repetitive_case()
            if make == "rep_nochain":
                monkeypatch.setenv("PHY_CHAIN", "0")
        elif make == "deep":
            case = cases.random_case(9, S=300, P=500, C=4, model="GTR", rooted=True)
        else:
            case = make()
            if make is cases.fluA_case:
                monkeypatch.setenv("PHY_CHAIN", "0")
    monkeypatch.setenv("PHY_STAGE_ORDER", str(1 << 40))
    plain = _class_engine(case, max_draws=3)
    monkeypatch.setenv("PHY_STAGE_ORDER", "0")
    porder = _class_engine(case, max_draws=3)
    monkeypatch.delenv("PHY_STAGE_ORDER")
    assert plain.class_info()["parent_order_levels"] == 0
    assert porder.class_info()["parent_order_levels"] >= 1, porder.class_info()
    a = porder.evaluate(case.blens, case.model_vec(), site_ll=True)
    b = plain.evaluate(case.blens, case.model_vec(), site_ll=True)
    _assert_rows_equal(a, b)
    check_case(case, porder, a)
    rng = np.random.default_rng(14)
    bl = case.blens[None, :] * rng.uniform(0.8, 1.2, (3, case.blens.size))
    mv = np.repeat(case.model_vec()[None], 3, axis=0)
    assert np.array_equal(porder.evaluate_rows(bl, mv), plain.evaluate_rows(bl, mv))
