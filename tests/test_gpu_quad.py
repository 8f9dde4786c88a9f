"""GPU: the quad sweep (csrc/quad_engine.inc) -- the pattern engine's path
for calls of <= 32 draws (a sampler's), a quad of lanes per (pattern,
category) column -- against the oracle and against the one / two column
sweeps (PHY_QUAD=0), through the C-ABI.

Tolerances as tests/test_gpu_parity.py: log L rel 1e-10, every gradient rel
1e-9 of its array's largest entry.
"""
import numpy as np
import pytest
import torch  # noqa: F401 -- torch's own HIP runtime must load before the engine's

from tests import cases
from tests.test_gpu_parity import RTOL_G, RTOL_LL, _close, check_case

pytestmark = pytest.mark.gpu


def _engine(case, max_draws=1, quad=True, monkeypatch=None):
    from phylostan_amd.engine import TreeLikelihood
    monkeypatch.setenv("PHY_QUAD", "1" if quad else "0")
    return TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C,
                          max_draws=max_draws)


def _draws(case, n, seed):
    rng = np.random.default_rng(seed)
    bl = case.blens[None, :] * rng.uniform(0.7, 1.4, (n, case.blens.size))
    mv = np.repeat(case.model_vec()[None], n, axis=0)
    return bl, mv


CASES = {
    "fluA": cases.fluA_case,
    "HCV": cases.hcv_case,
    "DS1": cases.ds1_case,
    "rand_C1_JC": lambda: cases.random_case(301, S=17, P=333, C=1, model="JC69"),
    "rand_C3_GTR": lambda: cases.random_case(302, S=40, P=500, C=3, model="GTR"),
    "rand_C16_HKY": lambda: cases.random_case(303, S=12, P=77, C=16, model="HKY"),
    "unrooted_C5": lambda: cases.random_case(304, S=33, P=250, C=5, model="GTR", rooted=False),
    "caterpillar": lambda: cases.random_case(305, S=60, P=150, C=4, model="HKY", caterpillar=True),
    "P1": lambda: cases.random_case(306, S=9, P=1, C=2, model="GTR"),
    "all_ambiguous": lambda: cases.random_case(307, S=10, P=90, C=2, model="GTR", ambiguous=1.0),
    # 94 blocks of 16 columns: a draw over more than 16 workgroups (qfin_kernel's batched slot sums)
    "many_blocks": lambda: cases.random_case(308, S=30, P=1500, C=4, model="GTR"),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_quad_single_eval_vs_oracle(name, monkeypatch):
    case = CASES[name]()
    eng = _engine(case, monkeypatch=monkeypatch)
    check_case(case, eng)


@pytest.mark.parametrize("name", ["fluA", "HCV", "DS1", "rand_C3_GTR", "unrooted_C5", "rand_C16_HKY", "many_blocks"])
@pytest.mark.parametrize("n", [4, 16, 32])
def test_quad_batch_rows_equal_column_sweeps(name, n, monkeypatch):
    """The sampler's shape (host buffers, n draws per call, full rows):
    every row of the quad sweep against the one/two-column sweeps' row."""
    case = CASES[name]()
    bl, mv = _draws(case, n, 11)
    quad = _engine(case, max_draws=n, monkeypatch=monkeypatch).evaluate_rows(bl, mv)
    ref = _engine(case, max_draws=n, quad=False, monkeypatch=monkeypatch).evaluate_rows(bl, mv)
    for k in range(n):
        assert abs(quad[k, 0] - ref[k, 0]) <= RTOL_LL * abs(ref[k, 0]), k
        _close(quad[k, 1:], ref[k, 1:], RTOL_G, "%s row %d" % (name, k))


def test_quad_rows_vs_oracle_and_deterministic(monkeypatch):
    case = cases.fluA_case()
    n = 8
    bl, mv = _draws(case, n, 5)
    eng = _engine(case, max_draws=n, monkeypatch=monkeypatch)
    a = eng.evaluate_rows(bl, mv)
    b = eng.evaluate_rows(bl, mv)
    assert np.array_equal(a, b), "quad sweep rows are not bitwise reproducible"
    for k in (0, 3, 7):
        c = cases.Case(case.name, case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, bl[k],
                       case.freqs, case.rates, case.rs, case.ps)
        ref = c.oracle()
        assert abs(a[k, 0] - ref["loglik"]) <= RTOL_LL * abs(ref["loglik"])
        _close(a[k, 1:1 + eng.B], ref["grad_blens"], RTOL_G, "grad_blens draw %d" % k)


def test_quad_compact_rows_and_async_pair(monkeypatch):
    case = cases.hcv_case()
    n = 4
    bl, mv = _draws(case, n, 9)
    eng = _engine(case, max_draws=n, monkeypatch=monkeypatch)
    eng.set_output(compact=True)
    ref = _engine(case, max_draws=n, quad=False, monkeypatch=monkeypatch)
    ref.set_output(compact=True)
    r = ref.evaluate_rows(bl, mv)
    eng.submit_rows(bl, mv)
    q = eng.wait_rows()
    for k in range(n):
        assert abs(q[k, 0] - r[k, 0]) <= RTOL_LL * abs(r[k, 0])
        _close(q[k, 1:], r[k, 1:], RTOL_G, "compact row %d" % k)


def test_quad_impossible_draw_is_minus_inf(monkeypatch):
    """L = 0 for one draw of a batch (a saturated branch between two
    incompatible tips): that row is -inf, its neighbours are untouched."""
    case = cases.random_case(310, S=6, P=40, C=2, model="JC69", ambiguous=0.0)
    n = 3
    bl, mv = _draws(case, n, 3)
    eng = _engine(case, max_draws=n, monkeypatch=monkeypatch)
    good = eng.evaluate_rows(bl, mv)
    bl2 = bl.copy()
    bl2[1] = 0.0  # every branch zero: P = I, tips disagree somewhere -> L = 0
    rows = eng.evaluate_rows(bl2, mv)
    assert rows[1, 0] == -np.inf
    assert np.array_equal(rows[0], good[0]) and np.array_equal(rows[2], good[2])


def test_prefer_latency_engine_is_the_quad_sweep_on_small_alignments(monkeypatch):
    """prefer_latency_engine keeps the pattern engine (its quad form for the
    sampler's 4-draw calls) when the automatic choice is the pattern sweep;
    its rows agree with the column sweep's."""
    case = cases.fluA_case()
    n = 4
    bl, mv = _draws(case, n, 21)
    eng = _engine(case, max_draws=n, monkeypatch=monkeypatch)
    assert eng.prefer_latency_engine() == "pattern"
    rows = eng.evaluate_rows(bl, mv)
    ref = _engine(case, max_draws=n, quad=False, monkeypatch=monkeypatch).evaluate_rows(bl, mv)
    for k in range(n):
        assert abs(rows[k, 0] - ref[k, 0]) <= RTOL_LL * abs(ref[k, 0])
        _close(rows[k, 1:], ref[k, 1:], RTOL_G, "row %d" % k)


def test_prefer_latency_engine_measures_class_against_pattern():
    """On an alignment the automatic choice sends to the class sweep, both
    engines are timed and the faster kept."""
    from phylostan_amd import synthetic
    from phylostan_amd.engine import TreeLikelihood
    pd, _ = synthetic.simulate(n_sites=60_000)  # the synthetic workload's tree and model, 60k sites
    eng = TreeLikelihood(pd.tipcodes, pd.weights, pd.peel0, True, "GTR", 4, max_draws=4)
    eng.set_engine("auto")
    assert eng.engine() == "class"
    name = eng.prefer_latency_engine(calls=8)
    assert set(eng.latency_probe) == {"pattern", "class"}
    assert name == min(eng.latency_probe, key=eng.latency_probe.get)


@pytest.mark.parametrize("name", ["fluA", "many_blocks"])
def test_quad_epilogue_handoffs_stress_bitwise(name, monkeypatch):
    """qfin_kernel's in-launch hand-offs to the draw's last workgroup (the
    HANDOFF note in phylo_hip.hip: write-through stores, drains, one ticket
    add, sc1 loads) under repetition: 10,000 back-to-back 4-draw sampler
    calls (compact rows, host buffers) in one process, every row bitwise
    equal to the first call's -- a stale hand-off anywhere shows as a
    differing row."""
    case = CASES[name]()
    n = 4
    bl, mv = _draws(case, n, 21)
    eng = _engine(case, max_draws=n, monkeypatch=monkeypatch)
    eng.set_output(compact=True)
    first = eng.evaluate_rows(bl, mv)
    bad = 0
    for _ in range(10000):
        bad += int(not np.array_equal(eng.evaluate_rows(bl, mv), first))
    assert bad == 0


@pytest.mark.parametrize("name", ["fluA", "HCV", "DS1", "rand_C1_JC", "rand_C3_GTR", "unrooted_C5", "many_blocks",
                                  "caterpillar", "balanced", "balanced64", "balanced128"])
@pytest.mark.parametrize("n", [1, 4, 16, 32])
def test_quad_multiwave_rows_bitwise_equal_one_wave(name, n, monkeypatch):
    """The multi-wave quad sweep (qmw_kernel: the post-order program split
    over up to 4 waves per category by the host list-scheduler, LDS slot
    hand-offs with flags) runs every step's arithmetic of the one-wave sweep
    and writes every dL/dP entry from the one wave owning its step: the rows,
    site log-likelihoods included, are bitwise PHY_QMW=0's."""
    make = {"caterpillar": lambda: cases.random_case(305, S=40, P=300, C=4, model="GTR", caterpillar=True),
            "balanced": lambda: cases.random_case(306, S=32, P=400, C=4, model="HKY"),
            # these two overflowed LDS with four waves per category and fell back to one wave (r05): the
            # plan now takes the most waves whose hand-off slots fit beside the matrix records (one-hot
            # and all-ones tips, as the reference's data: R = 5 record vectors; five more ambiguity
            # masks would make R = 9 and the 64-taxon records alone 145 KB of the 160)
            "balanced64": lambda: cases.random_case(306, S=64, P=400, C=4, model="HKY", ambiguous=0.0),
            "balanced128": lambda: cases.random_case(307, S=128, P=300, C=2, model="HKY", ambiguous=0.0),
            }.get(name, CASES.get(name))
    case = make()
    bl, mv = _draws(case, n, 41)
    out = {}
    for qmw in ("0", "1"):
        monkeypatch.setenv("PHY_QMW", qmw)
        eng = _engine(case, max_draws=n, monkeypatch=monkeypatch)
        plan = eng.quad_plan()
        if qmw == "0":
            assert plan["waves"] == 1 and plan["span"] == case.S - 1
        elif name in ("fluA", "HCV", "DS1", "balanced", "balanced64", "balanced128"):  # (a caterpillar has
            # nothing to run side by side)
            assert plan["waves"] >= 2 and plan["span"] < 0.75 * (case.S - 1), plan
        out[qmw] = eng.evaluate_rows(bl, mv)
        if n == 1:
            out[qmw + "s"] = eng.evaluate(case.blens, case.model_vec(), site_ll=True).site_ll
    assert np.array_equal(out["0"], out["1"])
    if n == 1:
        assert np.array_equal(out["0s"], out["1s"])


def test_quad_multiwave_stress_bitwise(monkeypatch):
    """2,000 back-to-back 4-draw fluA calls on the multi-wave sweep: every row
    bitwise the first call's (the slot hand-offs never read a stale value)."""
    import torch
    from phylostan_amd.engine import TreeLikelihood
    monkeypatch.setenv("PHY_QMW", "1")
    case = cases.fluA_case()
    eng = TreeLikelihood(case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, max_draws=4)
    bl, mv = _draws(case, 4, 43)
    ref = eng.evaluate_rows(bl, mv)
    d_bl = torch.tensor(bl, device="cuda:0")
    d_mv = torch.tensor(mv, device="cuda:0")
    d_out = torch.zeros((2000, 4, eng.outlen), dtype=torch.float64, device="cuda:0")
    s = torch.cuda.Stream()
    for k in range(2000):
        eng.evaluate_device(d_bl.data_ptr(), d_mv.data_ptr(), d_out[k].data_ptr(), 0, n_draws=4, stream=s.cuda_stream)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    assert np.array_equal(got, np.broadcast_to(ref, got.shape))
