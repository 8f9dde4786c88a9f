"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Tolerances (north_star: per-site log-likelihoods within 1e-6 relative of the
reference; we hold the HIP path to far tighter):
  per-site log L and total log L:  rel 1e-10 (+ abs 1e-12)
  gradients (dL/dP, blens, rs, ps, root freqs): rel 1e-9 of the largest
  entry's magnitude per array.
"""
import numpy as np
import pytest
import torch  # noqa: F401 -- torch's own HIP runtime must load before the engine's

from tests import cases

pytestmark = pytest.mark.gpu

RTOL_LL = 1e-10
RTOL_G = 1e-9


def _engine(case, max_draws=1, **kw):
    from phylostan_amd.engine import TreeLikelihood
    return TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C,
                          max_draws=max_draws, **kw)


def _close(a, b, rtol, what):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.max(np.abs(b)), 1e-300)
    err = np.max(np.abs(a - b)) / scale
    assert err <= rtol, "%s: max rel err %.3e > %.1e" % (what, err, rtol)


def check_case(case, eng=None, res=None):
    eng = eng or _engine(case)
    if res is None:
        res = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    ref = case.oracle()
    np.testing.assert_allclose(res.site_ll, ref["site_ll"], rtol=RTOL_LL, atol=1e-12)
    assert abs(res.loglik - ref["loglik"]) <= RTOL_LL * abs(ref["loglik"]) + 1e-12
    _close(res.dLdP, ref["dLdP"], RTOL_G, "dLdP")
    _close(res.grad_blens, ref["grad_blens"], RTOL_G, "grad_blens")
    _close(res.grad_rs, ref["grad_rs"], RTOL_G, "grad_rs")
    _close(res.grad_ps, ref["grad_ps"], RTOL_G, "grad_ps")
    _close(res.grad_freq_root, ref["grad_freq_root"], RTOL_G, "grad_freq_root")
    if case.model == "JC69":
        assert not np.any(res.grad_rates) and not np.any(res.grad_freqs)
    else:  # the device chain rule through Q vs the host one on the oracle's dL/dP
        from phylostan_amd import models
        gr, gf = models.q_param_gradients(ref["dLdP"], case.blens, case.rs, case.freqs, case.rates,
                                          ref["grad_freq_root"])
        _close(res.grad_rates, gr, 1e-8, "grad_rates")
        _close(res.grad_freqs, gf, 1e-8, "grad_freqs")
    return res


@pytest.mark.parametrize("seed,S,P,C,model,rooted,cat", [
    (1, 5, 1, 1, "JC69", True, False),       # single pattern
    (2, 12, 63, 3, "GTR", True, False),      # P < one block
    (3, 12, 130, 4, "HKY", True, False),     # ragged last block
    (4, 17, 257, 5, "GTR", False, False),    # unrooted, C=5 (+I-like)
    (5, 40, 200, 2, "GTR", True, True),      # caterpillar (deep tree)
    (6, 40, 200, 4, "JC69", False, True),    # unrooted caterpillar
    (7, 128, 300, 4, "GTR", True, False),    # synthetic-config taxa
    (8, 9, 100, 8, "HKY", True, False),      # C=8 -> 512-thread workgroups
])
def test_random_trees(seed, S, P, C, model, rooted, cat):
    check_case(cases.random_case(seed, S=S, P=P, C=C, model=model, rooted=rooted, caterpillar=cat))


def test_all_ambiguous_and_padding():
    case = cases.random_case(11, S=10, P=70, C=2, ambiguous=1.0)
    check_case(case)


@pytest.mark.parametrize("lds_budget,chunks", [(160 * 1024, 2), (80 * 1024, 4), (40000, None),
                                               (24000, None)])
def test_lds_plans(lds_budget, chunks):
    """Whole-program and chunked staging of P-matrices / dL/dP in LDS."""
    case = cases.fluA_case()
    eng = _engine(case)
    eng.set_tuning(0, 0, lds_budget)
    plan = eng.lds_plan()
    if chunks is not None:
        assert plan["n_chunks"] <= chunks
    else:
        assert plan["n_chunks"] > 1
    if lds_budget >= 40000:
        assert plan["lds_bytes"] <= lds_budget
    check_case(case, eng)


@pytest.mark.parametrize("mode", [1, 2], ids=["deep_lds", "deep_global"])
@pytest.mark.parametrize("cols", [1, 2])
@pytest.mark.parametrize("seed,S,P,C,model,rooted,cat,wg", [
    (41, 40, 300, 2, "GTR", True, False, 0),       # random topology: several deep entries
    (42, 128, 200, 4, "HKY", True, False, 3),      # synthetic-config taxa, persistent loop
    (43, 33, 140, 4, "GTR", False, False, 0),      # unrooted
])
def test_deep_stack_placement(mode, cols, seed, S, P, C, model, rooted, cat, wg):
    """The deep stack (operands waiting while a sibling subtree runs) in LDS
    or in the per-workgroup global region gives the oracle's answers."""
    case = cases.random_case(seed, S=S, P=P, C=C, model=model, rooted=rooted, caterpillar=cat)
    eng = _engine(case)
    eng.set_tuning(wg, cols, 0)
    eng.set_deep_stack(mode)
    depth = eng.program_info()["depth"]
    assert eng.lds_plan()["deep_lds_entries"] == (depth if mode == 1 else 0)
    check_case(case, eng)


@pytest.mark.parametrize("lds_budget", [60000, 80000, 100000])
def test_deep_stack_split(lds_budget):
    """Automatic plan under tight LDS: the outer deep entries in LDS, the
    inner ones in global memory (x operands read back from scratch slots)."""
    case = cases.random_case(44, S=128, P=300, C=4, model="GTR")
    eng = _engine(case)
    eng.set_tuning(0, 2, lds_budget)
    plan = eng.lds_plan()
    depth = eng.program_info()["depth"]
    assert 0 <= plan["deep_lds_entries"] <= depth
    print("budget", lds_budget, "depth", depth, plan)
    check_case(case, eng)


@pytest.mark.parametrize("cols", [1, 2])
@pytest.mark.parametrize("seed,S,P,C,model,rooted,cat,lds", [
    (31, 12, 130, 4, "HKY", True, False, 0),       # ragged: 130 = 128 + 2
    (32, 17, 257, 5, "GTR", False, False, 0),      # unrooted, odd C
    (33, 40, 300, 2, "GTR", True, True, 0),        # caterpillar
    (34, 64, 700, 4, "GTR", True, False, 40000),   # chunked, persistent loop
    (35, 9, 100, 8, "JC69", True, False, 0),       # 512-thread workgroups
])
def test_columns_per_lane(cols, seed, S, P, C, model, rooted, cat, lds):
    """One and two pattern columns per lane give the oracle's answers."""
    case = cases.random_case(seed, S=S, P=P, C=C, model=model, rooted=rooted, caterpillar=cat)
    eng = _engine(case)
    eng.set_tuning(3 if lds else 0, cols, lds or 160 * 1024)
    assert eng.lds_plan()["cols"] == cols
    check_case(case, eng)


@pytest.mark.parametrize("wg_budget", [0, 7])
def test_batched_draws_match_single(wg_budget):
    """Batched draws; wg_budget 7 = one workgroup per draw, whose dL/dP goes
    straight to the output rows across chunk flushes (no finalize sum)."""
    base = cases.fluA_case()
    rng = np.random.default_rng(3)
    n = 7
    eng = _engine(base, max_draws=n)
    if wg_budget:
        eng.set_tuning(wg_budget, 0, 0)
    blens = base.blens[None, :] * rng.uniform(0.5, 1.5, (n, 1))
    mvs = []
    for k in range(n):
        kappa = rng.uniform(2, 9)
        mvs.append(cases.models.model_vector(base.freqs, cases.models.hky_exchangeabilities(kappa),
                                             base.rs, base.ps))
    res = eng.evaluate_batch(blens, np.array(mvs), site_ll=True)
    for k in range(n):
        c = cases.Case("d%d" % k, base.tipcodes, base.weights, base.peel0, True, "HKY", 4, blens[k],
                       base.freqs, mvs[k][4:10], base.rs, base.ps)
        check_case(c, eng, res[k])


@pytest.mark.parametrize("make,engine", [(cases.fluA_case, "pattern"), (cases.hcv_case, "pattern"),
                                         (cases.fluA_case, "class"), (cases.hcv_case, "class")],
                         ids=["fluA-pattern", "HCV-pattern", "fluA-class", "HCV-class"])
def test_production_batch_every_row_vs_c_port(make, engine):
    """The bench's shape: 1,024 distinct parameter draws in ONE launch (the
    pattern sweep then runs one workgroup per draw with the finalize fused),
    every output row -- log L, branch / rate / mixture / root-frequency
    gradients, the device chain rule's exchangeability and frequency
    gradients, dL/dP -- against the C port at the parity bar."""
    from oracle import cpu
    from phylostan_amd import models
    base = make()
    n = 1024
    eng = _engine(base, max_draws=n)
    eng.set_engine(engine)
    rng = np.random.default_rng(17)
    blens = base.blens[None, :] * rng.uniform(0.5, 1.5, (n, base.blens.size))
    mvs = []
    for k in range(n):
        f = rng.dirichlet([30.0] * 4)
        r = (models.hky_exchangeabilities(rng.uniform(2.0, 9.0)) if base.model == "HKY"
             else base.rates * rng.uniform(0.7, 1.3, 6))
        rs, ps = models.weibull_site_rates(rng.uniform(0.2, 2.0), base.C)
        mvs.append(models.model_vector(f, r, rs, ps))
    mvs = np.array(mvs)
    rows = eng.evaluate_rows(blens, mvs)
    kind = {"JC69": 0, "HKY": 1, "GTR": 2}[base.model]
    for k in range(0, n, 37):  # 28 draws spread over the batch
        ref, _ = cpu.evaluate(base.tipcodes, base.weights, base.peel0, True, kind, mvs[k], blens[k], base.C)
        got = rows[k]
        assert abs(got[0] - ref[0]) <= RTOL_LL * abs(ref[0])
        B, C = eng.B, base.C
        o = 1 + B + 2 * C
        _close(got[1:o + 4], ref[1:o + 4], RTOL_G, "draw %d gradients" % k)
        _close(got[o + 4:o + 14], ref[o + 4:o + 14], 1e-8, "draw %d Q-parameter gradients" % k)
        _close(got[o + 14:], ref[o + 14:], RTOL_G, "draw %d dL/dP" % k)


@pytest.mark.parametrize("lds_budget", [0, 30000])
def test_persistent_workgroups_loop(lds_budget):
    """Fewer workgroups than pattern blocks: every workgroup loops (with the
    whole program or several chunks resident)."""
    case = cases.random_case(21, S=20, P=64 * 9 + 5, C=3)
    eng = _engine(case)
    eng.set_tuning(2, 0, lds_budget)
    check_case(case, eng)


def test_single_chunk_resident_for_small_tree():
    case = cases.random_case(22, S=10, P=300, C=2, model="HKY")
    eng = _engine(case)
    assert eng.lds_plan()["n_chunks"] == 1
    check_case(case, eng)


def test_deterministic():
    case = cases.hcv_case()
    eng = _engine(case)
    a = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    b = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    assert a.loglik == b.loglik
    assert np.array_equal(a.dLdP, b.dLdP) and np.array_equal(a.site_ll, b.site_ll)


def test_pruning_loglik_mirror():
    case = cases.ds1_case(1)
    eng = _engine(case)
    val, grad = eng.pruning_loglik(case.blens, case.model_vec())
    ref = case.oracle()
    assert abs(val - ref["loglik"]) <= 1e-10 * abs(ref["loglik"])
    _close(grad, ref["grad_blens"], RTOL_G, "grad")


def test_nonfinite_is_minus_inf():
    case = cases.random_case(5, S=6, P=10, C=1, model="JC69")
    eng = _engine(case)
    mv = case.model_vec()
    mv[10 + case.C:] = 0.0  # ps = 0 -> L = 0 -> log L = -inf
    res = eng.evaluate(case.blens, mv)
    assert res.loglik == -np.inf


@pytest.mark.parametrize("make,n", [(cases.hcv_case, 5), (cases.fluA_case, 3), (cases.fluA_case, 32)],
                         ids=["HCV-5", "fluA-3", "fluA-32"])
def test_host_eigensystems_bitwise_equal_device(make, n):
    """The small host-buffer path forms the eigensystems of up to 32 draws on
    the host (stage_small); the device path forms them on the GPU, inside the
    pmat waves for <= 32 draws.  Same operations in the same order without
    FMA contraction: every output row bit for bit."""
    base = make()
    rng = np.random.default_rng(29)
    from phylostan_amd import models
    eng = _engine(base, max_draws=n)
    bl = base.blens[None, :] * rng.uniform(0.6, 1.4, (n, base.blens.size))
    mv = []
    for _ in range(n):
        f = rng.dirichlet([20.0] * 4)
        r = (models.hky_exchangeabilities(rng.uniform(2.0, 9.0)) if base.model == "HKY"
             else base.rates * rng.uniform(0.6, 1.4, 6))
        rs, ps = models.weibull_site_rates(rng.uniform(0.2, 2.0), base.C)
        mv.append(models.model_vector(f, r, rs, ps))
    mv = np.array(mv)
    host = eng.evaluate_rows(bl, mv)
    d_bl = torch.tensor(bl, device="cuda:0")
    d_mv = torch.tensor(mv, device="cuda:0")
    d_out = torch.zeros((n, eng.outlen), dtype=torch.float64, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    eng.evaluate_device(d_bl.data_ptr(), d_mv.data_ptr(), d_out.data_ptr(), 0, n_draws=n, stream=stream)
    torch.cuda.synchronize()
    dev = d_out.cpu().numpy()
    assert np.array_equal(host, dev), "max |diff| %.3e" % np.max(np.abs(host - dev))


def test_submit_wait_equals_eval_and_guards_in_flight():
    """phy_eval_submit / phy_eval_wait give phy_eval's rows bit for bit; a
    second submit, phy_eval or phy_eval_device while one is in flight, and a
    wait with nothing submitted are refused."""
    from phylostan_amd._lib import PhyloHipError
    case = cases.hcv_case()
    eng = _engine(case, max_draws=4)
    rng = np.random.default_rng(12)
    bl = case.blens[None, :] * rng.uniform(0.8, 1.2, (3, 1))
    mv = np.repeat(case.model_vec()[None], 3, axis=0)
    ref = eng.evaluate_rows(bl, mv)
    eng.submit_rows(bl, mv)
    with pytest.raises(PhyloHipError):
        eng.submit_rows(bl, mv)
    with pytest.raises(PhyloHipError):
        eng.evaluate_rows(bl, mv)
    got = eng.wait_rows()
    assert np.array_equal(got, ref)
    with pytest.raises(PhyloHipError):
        eng.wait_rows()


def test_errors_are_loud():
    from phylostan_amd._lib import PhyloHipError
    case = cases.random_case(5, S=6, P=10, C=1, model="JC69")
    bad = case.peel0.copy()
    bad[0, 0] = 99
    with pytest.raises(PhyloHipError):
        cases.Case("bad", case.tipcodes, case.weights, bad, True, "JC69", 1, case.blens,
                   case.freqs, case.rates, case.rs, case.ps)
        _engine(cases.Case("bad", case.tipcodes, case.weights, bad, True, "JC69", 1, case.blens,
                           case.freqs, case.rates, case.rs, case.ps))
    eng = _engine(case)
    with pytest.raises(PhyloHipError):
        eng.evaluate_batch(np.tile(case.blens, (2, 1)), np.tile(case.model_vec(), (2, 1)))


@pytest.mark.parametrize("make", [cases.fluA_case, cases.hcv_case, cases.ds1_case],
                         ids=["fluA", "HCV", "DS1"])
def test_recomputed_cherries_bitwise(make):
    """Cherries rebuilt in the reverse half (not stored) give bit-identical
    outputs to the fully stored sweep, and match the oracle."""
    case = make()
    eng = _engine(case)
    assert eng.lds_plan()["recomputed"] > 0
    res = check_case(case, eng)
    eng.set_recompute(False)
    assert eng.lds_plan()["recomputed"] == 0
    ref = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    assert res.loglik == ref.loglik
    np.testing.assert_array_equal(res.site_ll, ref.site_ll)
    np.testing.assert_array_equal(res.dLdP, ref.dLdP)
    np.testing.assert_array_equal(res.grad_blens, ref.grad_blens)


def test_finalize_inside_sweep_matches_kernel(monkeypatch):
    """One workgroup per draw: the finalize folded into the sweep (default)
    and the separate finalize kernel (PHY_FIN=0) give bit-identical rows."""
    base = cases.fluA_case()
    rng = np.random.default_rng(5)
    n = 3
    blens = base.blens[None, :] * rng.uniform(0.7, 1.3, (n, 1))
    mv = np.repeat(base.model_vec()[None], n, axis=0)
    eng = _engine(base, max_draws=n)
    eng.set_tuning(n, 0, 0)  # one workgroup per draw
    r1 = eng.evaluate_batch(blens, mv, site_ll=True)
    monkeypatch.setenv("PHY_FIN", "0")
    eng2 = _engine(base, max_draws=n)
    eng2.set_tuning(n, 0, 0)
    r2 = eng2.evaluate_batch(blens, mv, site_ll=True)
    for a, b in zip(r1, r2):
        assert a.loglik == b.loglik
        np.testing.assert_array_equal(a.grad_blens, b.grad_blens)
        np.testing.assert_array_equal(a.grad_rs, b.grad_rs)
        np.testing.assert_array_equal(a.grad_ps, b.grad_ps)
        np.testing.assert_array_equal(a.grad_freq_root, b.grad_freq_root)
        np.testing.assert_array_equal(a.dLdP, b.dLdP)
    check_case(base, eng2)


@pytest.mark.parametrize("S,P,cat", [(400, 300, False), (300, 200, True)], ids=["random400", "caterpillar300"])
def test_large_trees(S, P, cat):
    """Hundreds of taxa: deep stacks, many LDS chunks, long rebuild chains."""
    case = cases.random_case(61, S=S, P=P, C=4, model="GTR", caterpillar=cat)
    eng = _engine(case)
    plan = eng.lds_plan()
    assert plan["n_chunks"] > 1
    check_case(case, eng)


def test_every_ambiguity_mask():
    """All 15 non-empty 4-bit masks in the data: 15 record vectors per matrix."""
    case = cases.random_case(62, S=20, P=400, C=3, model="HKY")
    rng = np.random.default_rng(62)
    codes = rng.integers(1, 16, size=case.tipcodes.shape).astype(np.uint8)
    case = cases.Case("allmasks", codes, case.weights, case.peel0, True, "HKY", 3, case.blens, case.freqs,
                      case.rates, case.rs, case.ps)
    check_case(case)


@pytest.mark.parametrize("C", [9, 16])
def test_many_categories(C):
    """C > 8 rate categories: one column per lane, C waves per workgroup."""
    case = cases.random_case(63, S=24, P=150, C=C, model="GTR")
    eng = _engine(case)
    assert eng.lds_plan()["cols"] == 1
    check_case(case, eng)


@pytest.mark.parametrize("engine", ["pattern", "class"])
def test_compact_output_rows(engine):
    """phy_set_output(compact): the rows stop after the model-parameter
    gradients; every value equals the full row's bit for bit."""
    case = cases.hcv_case()
    eng = _engine(case, max_draws=3)
    eng.set_engine(engine)
    rng = np.random.default_rng(9)
    bl = case.blens[None, :] * rng.uniform(0.8, 1.2, (3, 1))
    mv = np.repeat(case.model_vec()[None], 3, axis=0)
    full = eng.evaluate_batch(bl, mv)
    n_full = eng.outlen
    eng.set_output(compact=True)
    assert eng.outlen == n_full - 16 * case.C * eng.B == 1 + eng.B + 2 * case.C + 14
    comp = eng.evaluate_batch(bl, mv)
    for a, b in zip(full, comp):
        assert b.dLdP is None and a.loglik == b.loglik
        for k in ("grad_blens", "grad_rs", "grad_ps", "grad_freq_root", "grad_rates", "grad_freqs"):
            np.testing.assert_array_equal(getattr(a, k), getattr(b, k))
    check_case(case, eng.__class__(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C))


def test_tuning_grows_workgroup_regions_past_create():
    """phy_set_tuning with a workgroup budget beyond what phy_create sized
    the per-workgroup regions for grows them (round 1 refused with
    PHY_ERANGE); results equal the default plan's."""
    case = cases.random_case(91, S=30, P=5000, C=4, model="GTR")
    eng = _engine(case, max_draws=2)
    ref = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    eng.set_tuning(4096, 1, 0)  # 1 column per lane: up to 79 blocks per draw
    got = eng.evaluate(case.blens, case.model_vec(), site_ll=True)
    np.testing.assert_allclose(got.site_ll, ref.site_ll, rtol=RTOL_LL, atol=1e-12)
    _close(got.dLdP, ref.dLdP, RTOL_G, "dLdP")
    check_case(case, eng, got)



@pytest.mark.parametrize("engine", ["pattern", "class"])
@pytest.mark.parametrize("S,rooted,max_draws", [(3, True, 1), (3, False, 1), (4, False, 1), (3, True, 4096),
                                                (3, False, 4096)],
                         ids=["S3-rooted", "S3-unrooted", "S4-unrooted", "S3-rooted-batched", "S3-unrooted-batched"])
def test_minimal_trees(engine, S, rooted, max_draws):
    """The smallest trees the boundary accepts (S = 3; an unrooted tree's root
    then has a tip child on the merged branch), on every engine, with the
    sampler's one-column plan (max_draws 1) and the batched two-column plan."""
    case = cases.random_case(31 + S, S=S, P=7, C=2, model="GTR", rooted=rooted)
    eng = _engine(case, max_draws=max_draws)
    eng.set_engine(engine)
    check_case(case, eng)


@pytest.mark.parametrize("engine", ["pattern", "class"])
def test_zero_and_saturated_branches_and_zero_weights(engine):
    """Internal branch lengths of zero (P = I, dP/dt = Q; a zero tip branch
    would make patterns impossible) and branches of 40 substitutions (P at
    the stationary distribution, vanishing gradients), and patterns of weight
    zero (present in the alignment, no contribution)."""
    case = cases.random_case(41, S=16, P=90, C=3, model="GTR")
    case.blens[case.S::3] = 0.0  # branch b sits above node b + 1: b >= S are internal
    case.blens[1::5] = 40.0
    case.weights[::7] = 0.0
    ref = case.oracle()
    assert np.isfinite(ref["loglik"])
    eng = _engine(case)
    eng.set_engine(engine)
    check_case(case, eng)


@pytest.mark.parametrize("engine", ["pattern", "class"])
@pytest.mark.parametrize("max_draws", [8, 4096], ids=["one-column", "batched"])
def test_impossible_draw_inside_a_batch(engine, max_draws):
    """One draw of a batch with L = 0 (mixture weights all zero) comes back
    as -inf; its neighbours' rows equal their single-draw rows bit for bit
    (nothing of the impossible draw leaks through shared slots or sums)."""
    case = cases.random_case(51, S=12, P=80, C=2, model="HKY")
    eng = _engine(case, max_draws=max_draws)
    eng.set_engine(engine)
    n = 5
    bl = np.repeat(case.blens[None], n, axis=0) * np.linspace(0.8, 1.2, n)[:, None]
    mv = np.repeat(case.model_vec()[None], n, axis=0)
    mv[2, 10 + case.C:] = 0.0
    rows = eng.evaluate_rows(bl, mv)
    assert rows[2, 0] == -np.inf
    for k in (0, 1, 3, 4):
        one = eng.evaluate_rows(bl[k:k + 1], mv[k:k + 1])[0]
        assert np.array_equal(rows[k], one), k
        assert np.isfinite(rows[k]).all()


def test_retired_resident_engine_is_refused():
    """Engine 3 (round 3's resident class sweep) is retired: phy_set_engine
    refuses it with PHY_EINVAL and a message naming the replacement."""
    from phylostan_amd._lib import PhyloHipError
    case = cases.fluA_case()
    eng = _engine(case, max_draws=4)
    with pytest.raises(PhyloHipError, match="retired"):
        eng.set_engine(3)
    assert eng.engine() == "pattern"

