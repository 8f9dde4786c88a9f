"""CPU: the C-ABI library builds, loads and exports exactly what
include/phylo_hip.h (the consumer boundary) and include/phylo_hip_diag.h
(planning / introspection) declare; without a GPU the product fails loudly."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "phylo_hip.h")
DIAG_HEADER = os.path.join(ROOT, "include", "phylo_hip_diag.h")


def declared_functions(headers=(HEADER, DIAG_HEADER)):
    names = set()
    for h in headers:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names.update(re.findall(r"\b(phy_[a-z_]+)\s*\(", text))
    return sorted(names)


def test_header_declares_the_boundary():
    names = declared_functions((HEADER,))
    assert names == sorted(["phy_create", "phy_create_multi", "phy_destroy", "phy_last_error", "phy_num_branches",
                            "phy_output_len", "phy_eval", "phy_eval_device", "phy_eval_submit", "phy_eval_wait",
                            "phy_pruning_loglik", "phy_sync", "phy_set_output"])
    diag = declared_functions((DIAG_HEADER,))
    assert not set(names) & set(diag)


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


def test_stale_build_is_refused(tmp_path, monkeypatch):
    """A library lacking an entry point is refused at load, even when it is a
    PHYLO_HIP_LIB variant; only PHYLO_HIP_AB=1 (A/B runs) binds a partial one."""
    import subprocess
    from phylostan_amd import _lib
    src = tmp_path / "stale.c"
    src.write_text("int phy_create(void) { return 0; }\n")
    so = tmp_path / "stale.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    monkeypatch.setenv("PHYLO_HIP_LIB", str(so))
    monkeypatch.delenv("PHYLO_HIP_AB", raising=False)
    with pytest.raises(_lib.PhyloHipError, match="stale build"):
        _lib.load(str(so))
    monkeypatch.setenv("PHYLO_HIP_AB", "1")
    lib = _lib.load(str(so))
    assert hasattr(lib, "phy_create")


def test_torch_after_engine_is_a_clear_error():
    """Run in a fresh interpreter: by default the engine loads without torch
    (a non-torch consumer pays nothing), a probe still finds torch, and a
    later `import torch` raises the guard's ImportError instead of leaving
    torch without a GPU; with PHYLO_WITH_TORCH=1 load() imports torch first,
    so the order is right by construction."""
    import subprocess
    import sys
    from phylostan_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("HIP library not built")
    code = ("import sys, importlib.util; sys.path.insert(0, %r)\n"
            "from phylostan_amd import _lib\n"
            "_lib.load()\n"
            "print('torch loaded before engine:', 'torch' in sys.modules)\n"
            "print('probe finds torch:', importlib.util.find_spec('torch') is not None)\n"
            "try:\n"
            "    import torch\n"
            "    print('import ok')\n"
            "except ImportError as e:\n"
            "    print('guard:', 'imported after' in str(e))\n") % ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("PHYLO_WITH_TORCH", "PHYLO_NO_TORCH")}
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert "torch loaded before engine: False" in out.stdout, out.stdout + out.stderr
    assert "probe finds torch: True" in out.stdout, out.stdout + out.stderr
    assert "guard: True" in out.stdout, out.stdout + out.stderr
    env["PHYLO_WITH_TORCH"] = "1"
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert "torch loaded before engine: True" in out.stdout, out.stdout + out.stderr
    assert "import ok" in out.stdout, out.stdout + out.stderr
