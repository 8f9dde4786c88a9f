"""``python -m phylostan_amd build|run|parse``: flags, output files and their
formats (phylostan/phylostan.py:15-335, utils.py:193-409), on the CPU with the
oracle stand-in as the likelihood (the GPU run of the same CLI is in
tests/test_gpu_inference.py)."""
import json
import os

import numpy as np
import pytest

from phylostan_amd import cli, stan_io
from tests import fixture_files
from tests.oracle_backend import OracleLikelihood


def _run(argv, **kw):
    import argparse
    parser = argparse.ArgumentParser()
    sub = parser.add_subparsers()
    cli.create_run_parser(sub).set_defaults(func=cli.run)
    arg = parser.parse_args(["run"] + argv)
    lines = []
    post = cli.run(arg, likelihood_factory=OracleLikelihood, log=lines.append, **kw)
    return post, lines


def test_build_writes_model_description(tmp_path):
    script = str(tmp_path / "m.json")
    assert cli.main(["build", "-s", script, "-m", "HKY", "-C", "4", "--clock", "strict", "--estimate_rate",
                     "--coalescent", "constant", "--heterochronous"]) == 0
    doc = json.load(open(script))
    assert doc["options"]["model"] == "HKY" and doc["options"]["categories"] == 4


def test_run_vb_outputs(tmp_path, capsys):
    t, a = fixture_files.write_random_dataset(str(tmp_path), seed=1, S=6, sites=50)
    out = str(tmp_path / "rand")
    post, lines = _run(["-s", str(tmp_path / "x.stan"), "-m", "HKY", "-C", "2", "--clock", "strict",
                        "--estimate_rate", "--coalescent", "constant", "--heterochronous", "-t", t, "-i", a,
                        "-o", out, "-S", "7", "--iter", "300", "--elbo_samples", "20", "--samples", "50",
                        "--tol_rel_obj", "0.01"])
    assert any("Begin stochastic gradient ascent." in s for s in lines)
    assert any(s.startswith("   100") or s.startswith("  100") for s in lines)
    header, data = stan_io.read_samples(out)
    assert header[0] == "lp__" and header[1:4] == ["wshape", "props.1", "props.2"]
    assert "heights.5" in header and "rs.2" in header and "freqs.4" in header
    assert data.shape == (51, len(header)) and np.all(data[:, 0] == 0)
    diag = open(out + ".diag").read().splitlines()
    rows = [r for r in diag if not r.startswith("#")]
    assert rows[0] == "iter,time_in_seconds,ELBO" and rows[1].startswith("100,")
    trees = open(out + ".trees").read()
    assert trees.startswith("#NEXUS\nBegin trees;\nTranslate\n1 t") and trees.count("tree ") == 51
    assert "[&height=" in trees and ",rate=" in trees and trees.endswith("END;")
    printed = capsys.readouterr().out
    assert "Strict clock (rate) mean:" in printed and "Root height mean:" in printed


def test_run_nuts_two_chains_and_parse(tmp_path, capsys):
    t, a = fixture_files.write_random_dataset(str(tmp_path), seed=2, S=5, sites=40, hetero=False)
    out = str(tmp_path / "nuts")
    post, lines = _run(["-s", str(tmp_path / "x.stan"), "-m", "JC69", "-t", t, "-i", a, "-o", out, "-a", "nuts",
                        "--chains", "2", "--iter", "40", "-S", "3"])
    for c in range(2):
        path = out + "_%d.csv" % c
        header, data = stan_io.read_samples(path)
        assert header[:7] == ["lp__"] + stan_io.NUTS_COLUMNS
        assert header[7] == "blens.1" and data.shape[0] == 20
        txt = open(path).read()
        assert "# Adaptation terminated" in txt and "# Diagonal elements of inverse mass matrix:" in txt
        assert os.path.exists(out + "_%d.trees" % c)
    capsys.readouterr()
    cli.main(["parse", "--samples", out + "_0.csv", "-t", t, "-o", str(tmp_path / "p.trees")])
    printed = capsys.readouterr().out
    assert "Tree length mean:" in printed
    assert open(str(tmp_path / "p.trees")).read().count("tree ") == 20


def test_run_relaxed_clock_vb(tmp_path, capsys):
    """--clock ucln --estimate_rate: substrates in the sample CSV, per-branch
    rates in the trees file (utils.py:229-245)."""
    t, a = fixture_files.write_random_dataset(str(tmp_path), seed=3, S=6, sites=50)
    out = str(tmp_path / "ucln")
    post, lines = _run(["-s", str(tmp_path / "x.stan"), "-m", "JC69", "--clock", "ucln", "--estimate_rate",
                        "--coalescent", "constant", "--heterochronous", "-t", t, "-i", a,
                        "-o", out, "-S", "5", "--iter", "200", "--elbo_samples", "10", "--samples", "20",
                        "--tol_rel_obj", "0.01"])
    header, data = stan_io.read_samples(out)
    assert "substrates.10" in header and "ucln_stdev" in header
    assert data.shape == (21, len(header))
    trees = open(out + ".trees").read()
    assert trees.count("tree ") == 21 and ",rate=" in trees
    capsys.readouterr()


def test_unsupported_options_fail_loudly(tmp_path):
    t, a = fixture_files.write_random_dataset(str(tmp_path), seed=1, S=5, sites=20)
    with pytest.raises((SystemExit, ValueError)):
        _run(["-s", "x", "-t", t, "-i", a, "-o", str(tmp_path / "o"), "--clock", "acln"])  # needs --estimate_rate
    with pytest.raises(SystemExit):
        _run(["-s", "x", "-t", t, "-i", a, "-o", str(tmp_path / "o"), "--geo"])
    with pytest.raises(SystemExit):
        _run(["-s", "x", "-t", t, "-i", a, "-o", str(tmp_path / "o"), "-a", "hmc"])
