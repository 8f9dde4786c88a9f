"""CPU: the C-ABI library builds, loads and exports exactly what
include/phylo_hip.h declares; without a GPU the product fails loudly."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "phylo_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(phy_[a-z_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("phy_create", "phy_destroy", "phy_eval", "phy_eval_device", "phy_pruning_loglik",
                     "phy_last_error"):
        assert required in names


def test_library_exports_every_declared_symbol():
    from phylostan_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("HIP library not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding covers the whole product surface
    assert set(_lib.SIGNATURES) <= set(declared_functions())


def test_no_gpu_means_loud_failure():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from phylostan_amd import _lib
    from phylostan_amd.engine import TreeLikelihood
    from tests import cases
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("HIP library not built")
    case = cases.kat_case(cases.load_kat()["points"][0])
    with pytest.raises(_lib.PhyloHipError):
        TreeLikelihood(case.tipcodes, case.weights, case.peel0, True, "JC69", 1)


def test_missing_library_is_an_error(tmp_path):
    from phylostan_amd import _lib
    with pytest.raises(_lib.PhyloHipError):
        _lib.load(str(tmp_path / "nope.so"))
