"""GPU: a C++ host linked against libphylo_hip.so through include/phylo_hip.h
alone (tests/abi_consumer.cpp, built by __graft_entry__.build()), in the shape
of the reference's Stan external function (eigen/prune_stan.hpp:9-17, the
drop-in of INTEGRATION.md section 1), against the oracle: fluA HKY+W4 (the
bench config) and DS1 JC69 unrooted, one context and a two-shard
phy_create_multi handle."""
import os
import subprocess

import numpy as np
import pytest

from tests import cases

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "abi_consumer")
MODEL_IDS = {"JC69": 0, "HKY": 1, "GTR": 2}


def _write_input(path, case, draws):
    S, P = case.tipcodes.shape
    with open(path, "w") as fp:
        fp.write("%d %d %d %d %d %d\n" % (S, P, case.C, int(case.rooted), MODEL_IDS[case.model], len(draws)))
        fp.write(" ".join(str(int(v)) for v in case.tipcodes.ravel()) + "\n")
        fp.write(" ".join(repr(float(v)) for v in case.weights) + "\n")
        fp.write(" ".join(str(int(v)) for v in case.peel0.ravel()) + "\n")
        for bl, mv in draws:
            fp.write(" ".join(repr(float(v)) for v in bl) + "\n")
            fp.write(" ".join(repr(float(v)) for v in mv) + "\n")


def _parse(out, B):
    dbl, var = {}, {}
    misuse = None
    for line in out.splitlines():
        f = line.split()
        if f[0] == "double":
            dbl[int(f[1])] = float(f[2])
        elif f[0] == "var":
            var[int(f[1])] = np.array([float(x) for x in f[2:]])
            assert var[int(f[1])].size == 1 + B
        elif f[0] == "misuse":
            misuse = f[1:]
    return dbl, var, misuse


@pytest.mark.parametrize("name", ["fluA", "DS1"])
@pytest.mark.parametrize("mode", ["single", "multi2"])
def test_cpp_consumer_matches_oracle(tmp_path, name, mode):
    if not os.path.exists(BIN):
        pytest.fail("tests/abi_consumer was not built (run __graft_entry__.build())")
    case = cases.fluA_case() if name == "fluA" else cases.ds1_case()
    rng = np.random.default_rng(7)
    draws = [(case.blens, case.model_vec())]
    bl2 = case.blens * rng.uniform(0.8, 1.25, case.blens.size)
    draws.append((bl2, case.model_vec()))
    inp = tmp_path / "in.txt"
    _write_input(inp, case, draws)
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = os.path.join(ROOT, "phylostan_amd") + ":" + env.get("LD_LIBRARY_PATH", "")
    r = subprocess.run([BIN, str(inp), mode], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    B = case.blens.size
    dbl, var, misuse = _parse(r.stdout, B)
    assert misuse == ["nan", "msg"]
    for d, (bl, _) in enumerate(draws):
        c = cases.Case(case.name, case.tipcodes, case.weights, case.peel0, case.rooted, case.model, case.C, bl,
                       case.freqs, case.rates, case.rs, case.ps)
        ref = c.oracle()
        assert abs(dbl[d] - ref["loglik"]) <= 1e-10 * abs(ref["loglik"])
        assert var[d][0] == dbl[d]  # both overloads: one evaluation path
        g = var[d][1:]
        assert np.max(np.abs(g - ref["grad_blens"])) <= 1e-9 * np.max(np.abs(ref["grad_blens"]))
