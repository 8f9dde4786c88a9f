"""The committed bench lines (profiles/r0N_*_bench.json, the latest round's) keep bench.py's
contract: the driver's keys, a roofline whose fraction is its own
achieved / peak and whose achieved rate is the algorithmic bytes over the
kernel's average launch, a cpu_baseline with the fields the task names, and
the metric BASELINE.json names.  No GPU: these read the files only."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
def latest(kind):
    """The newest round's committed line of this kind (r06_..., else r05_..., r04_..., r03_...)."""
    for r in ("r06", "r05", "r04", "r03"):
        if os.path.exists(os.path.join(ROOT, "profiles", "%s_%s" % (r, kind))):
            return "%s_%s" % (r, kind)
    raise FileNotFoundError(kind)


LINES = [latest(k) for k in ("fluA_bench.json", "HCV_bench.json", "DS1_bench.json", "synthetic_class_bench.json")]
KEYS = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"]


def check_roofline(rf):
    """The pattern sweep is priced against the fp64 vector roof with SURVEY.md
    8d's algorithmic flops (its HBM view beside it); the class sweep against
    HBM with the algorithmic bytes.  Either way achieved = algorithmic work of
    one launch / the kernel's average launch, frac = achieved / peak."""
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"], rel=1e-12)
    t = rf["kernel_avg_ms"] * 1e-3
    if rf["bound"] == "fp64-vector":
        assert rf["unit"] == "TFLOP/s" and rf["peak"] == 78.6
        assert rf["achieved"] == pytest.approx(rf["algorithmic_flops_per_launch"] / t / 1e12, rel=1e-9)
        hbm = rf["hbm"]
        assert hbm["unit"] == "GB/s" and hbm["peak"] == 8000.0
        assert hbm["achieved"] == pytest.approx(hbm["algorithmic_bytes_per_launch"] / t / 1e9, rel=1e-9)
        assert hbm["frac"] == pytest.approx(hbm["achieved"] / hbm["peak"], rel=1e-12)
    else:
        assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
        assert rf["achieved"] == pytest.approx(rf["algorithmic_bytes_per_launch"] / t / 1e9, rel=1e-9)


def last_line(name):
    with open(os.path.join(ROOT, "profiles", name)) as f:
        return json.loads(f.read().strip().splitlines()[-1])


@pytest.mark.parametrize("name", LINES)
def test_committed_bench_line_keeps_the_contract(name):
    d = last_line(name)
    for k in KEYS:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["dtype"] == "f64"
    assert "workload" in d["config"]
    check_roofline(d["roofline"])
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] in ("port", "reference") and cb["unit"] == d["unit"]


def test_headline_metric_is_baselines():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    d = last_line(latest("fluA_bench.json"))
    assert d["metric"] == base["metric"]
    assert d["nominal_check"]["ok"] is True
    # value: draws per step over the step time
    assert d["value"] == pytest.approx(d["config"]["draws_per_step"] / (d["ms_per_step"] * 1e-3), rel=1e-9)


def test_pmc_traffic_belongs_to_the_committed_lines():
    """A line reports the PMC traffic of its own kernel source only: equal to
    the committed record when the sources match, null otherwise (bench.py
    never prices a launch with another build's counters)."""
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        pmc = json.load(f)
    d = last_line(latest("fluA_bench.json"))
    if d["kernel_source"] == pmc["kernel_source"]:
        assert d["roofline"]["traffic"] == pytest.approx(pmc["per_launch_bytes"]["fluA:8192:pattern"], rel=1e-12)
    else:
        assert d["roofline"]["traffic"] is None


def test_default_line_carries_the_synthetic_record():
    """bench.py's default run (the driver's BENCH line) carries BASELINE
    config 4 -- the 128 x 1M synthetic alignment, one draw per step -- timed
    in the same process, with its own roofline, CPU baseline and nominal check
    (VERDICT r04 next-round item 1)."""
    d = last_line(latest("fluA_bench.json"))
    if "synthetic" not in d:
        pytest.skip("the committed fluA line predates the synthetic sub-record")
    sy = d["synthetic"]
    for k in KEYS:
        assert k in sy, k
    for k in ("allreduce", "nominal_check", "multidev", "program"):
        assert k in sy, k
    assert sy["dtype"] == "f64" and sy["unit"] == "evals/s" and sy["scaling"] == "strong"
    assert sy["config"]["draws_per_step"] == 1 and sy["config"]["taxa"] == 128
    assert sy["value"] == pytest.approx(1.0 / (sy["ms_per_step"] * 1e-3), rel=1e-9)
    check_roofline(sy["roofline"])
    assert sy["nominal_check"]["ok"] is True
    assert sy["nominal_check"]["rel_err"] <= 1e-10 and sy["nominal_check"]["grad_blens_max_rel_err"] <= 1e-8
    cb = sy["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["unit"] == "evals/s"
    if sy["n_gpus"] == 1:
        assert sy["multidev"] is None


def test_default_line_reports_the_one_draw_sampler_call():
    d = last_line(latest("fluA_bench.json"))
    sl = d["sampler_latency"]
    if "pattern_us_per_call_1draw" not in sl:
        pytest.skip("the committed fluA line predates the 1-draw figure")
    assert 0 < sl["pattern_us_per_call_1draw"] < 1e4
    assert d["draws_100"] is not None


def _check_counted(hbm, traffic, alg, kern_ms):
    if traffic is None:
        assert hbm["counted_gbps"] is None and hbm["counted_frac"] is None
        return
    g = traffic / (kern_ms * 1e-3) / 1e9
    assert hbm["counted_gbps"] == pytest.approx(g, rel=1e-12)
    assert hbm["counted_frac"] == pytest.approx(g / 8000.0, rel=1e-12)
    assert hbm["traffic_over_algorithmic"] == pytest.approx(traffic / alg, rel=1e-12)
    assert ("below" in hbm["counted_note"]) == (traffic < alg)


def test_default_line_reports_counted_hbm_and_all_thread_baselines():
    """the rocprof-counted HBM rate (PMC bytes per launch
    over the kernel's average launch) beside the algorithmic one, for fluA and
    synthetic, a note when counted bytes are below algorithmic, and the
    synthetic record's OpenMP CPU baseline on the job's threads."""
    d = last_line(latest("fluA_bench.json"))
    rf = d["roofline"]
    if "counted_gbps" not in rf.get("hbm", {}):
        pytest.skip("the committed fluA line predates the counted HBM rate")
    _check_counted(rf["hbm"], rf["traffic"], rf["hbm"]["algorithmic_bytes_per_launch"], rf["kernel_avg_ms"])
    sy = d["synthetic"]
    srf = sy["roofline"]
    _check_counted(srf["hbm"], srf["traffic"], srf["algorithmic_bytes_per_launch"], srf["kernel_avg_ms"])
    mt = sy["cpu_baseline_all_threads"]
    assert mt["kind"] == "port" and mt["cores"] > 1 and mt["unit"] == "evals/s" and mt["value"] > 0
    assert d["cpu_baseline_all_threads"]["cores"] == mt["cores"]
