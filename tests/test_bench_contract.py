"""The committed bench lines (profiles/r03_*_bench.json) keep bench.py's
contract: the driver's keys, a roofline whose fraction is its own
achieved / peak and whose achieved rate is the algorithmic bytes over the
kernel's average launch, a cpu_baseline with the fields the task names, and
the metric BASELINE.json names.  No GPU: these read the files only."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINES = ["r03_fluA_bench.json", "r03_HCV_bench.json", "r03_DS1_bench.json", "r03_synthetic_class_bench.json"]
KEYS = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"]


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
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"], rel=1e-12)
    # achieved = algorithmic bytes of one launch / the kernel's average launch
    assert rf["achieved"] == pytest.approx(rf["algorithmic_bytes_per_launch"] / (rf["kernel_avg_ms"] * 1e-3) / 1e9,
                                           rel=1e-9)
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] in ("port", "reference") and cb["unit"] == d["unit"]


def test_headline_metric_is_baselines():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    d = last_line("r03_fluA_bench.json")
    assert d["metric"] == base["metric"]
    assert d["nominal_check"]["ok"] is True
    # value: draws per step over the step time
    assert d["value"] == pytest.approx(d["config"]["draws_per_step"] / (d["ms_per_step"] * 1e-3), rel=1e-9)


def test_pmc_traffic_belongs_to_the_committed_lines():
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        pmc = json.load(f)
    d = last_line("r03_fluA_bench.json")
    assert d["kernel_source"] == pmc["kernel_source"]
    assert d["roofline"]["traffic"] == pytest.approx(pmc["per_launch_bytes"]["fluA:8192:pattern"], rel=1e-12)
