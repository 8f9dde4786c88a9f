"""ctypes binding of the C-ABI in ``include/phylo_hip.h``.

This is the Python-side binding a maintainer would add to the reference in
place of its Stan external-function plumbing (``eigen/util.py:113-129`` /
``eigen/prune_stan.hpp``): the shared library is loaded once, every entry
point gets an explicit signature, and a missing library is a hard error --
there is no CPU fallback in the product path.
"""
import ctypes
import importlib.abc
import importlib.machinery
import importlib.util
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PHYLO_HIP_LIB") or os.path.join(_HERE, "libphylo_hip.so")

PHY_JC69, PHY_HKY, PHY_GTR = 0, 1, 2

_lib = None

_c_double_p = ctypes.POINTER(ctypes.c_double)
_c_int_p = ctypes.POINTER(ctypes.c_int)

# name -> (restype, argtypes)
SIGNATURES = {
    "phy_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                  ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "phy_create_multi": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "phy_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "phy_last_error": (ctypes.c_char_p, []),
    "phy_num_branches": (ctypes.c_int, [ctypes.c_void_p]),
    "phy_output_len": (ctypes.c_int, [ctypes.c_void_p]),
    "phy_program_info": (ctypes.c_int, [ctypes.c_void_p, _c_int_p, _c_int_p, _c_int_p, _c_int_p]),
    "phy_eval": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_void_p]),
    "phy_eval_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "phy_eval_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "phy_eval_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "phy_pruning_loglik": (ctypes.c_double, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p]),
    "phy_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "phy_timing_start": (ctypes.c_int, [ctypes.c_void_p]),
    "phy_timing_read": (ctypes.c_int, [ctypes.c_void_p, _c_double_p, _c_int_p]),
    "phy_set_tuning": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "phy_lds_plan": (ctypes.c_int, [ctypes.c_void_p, _c_int_p, _c_int_p, _c_int_p]),
    "phy_columns_per_lane": (ctypes.c_int, [ctypes.c_void_p]),
    "phy_set_deep_stack": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "phy_deep_stack_in_lds": (ctypes.c_int, [ctypes.c_void_p]),
    "phy_set_recompute": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "phy_recomputed_partials": (ctypes.c_int, [ctypes.c_void_p]),
    "phy_set_engine": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "phy_set_output": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "phy_engine": (ctypes.c_int, [ctypes.c_void_p]),
    "phy_class_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), _c_int_p, _c_int_p,
                                      ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong),
                                      _c_int_p, _c_int_p]),
    "phy_class_clades": (ctypes.c_int, [ctypes.c_void_p, _c_int_p, _c_int_p, ctypes.POINTER(ctypes.c_longlong)]),
    "phy_class_chain": (ctypes.c_int, [ctypes.c_void_p, _c_int_p, _c_int_p, _c_int_p]),
    "phy_quad_plan": (ctypes.c_int, [ctypes.c_void_p, _c_int_p, _c_int_p, _c_int_p]),
    "phy_class_fused": (ctypes.c_int, [ctypes.c_void_p, _c_int_p, _c_int_p, _c_int_p]),
}


class PhyloHipError(RuntimeError):
    pass


_GUARD_MSG = (
    "phylostan_amd: torch imported after libphylo_hip.so was loaded; torch's bundled HIP runtime cannot "
    "initialise the GPU after the engine's runtime holds it.  Import torch before phylostan_amd's engine, "
    "or set PHYLO_WITH_TORCH=1 so that loading the engine imports torch first.")


class _GuardLoader(importlib.abc.Loader):
    def create_module(self, spec):
        raise ImportError(_GUARD_MSG)

    def exec_module(self, module):  # never reached
        raise ImportError(_GUARD_MSG)


class _TorchAfterEngineGuard(importlib.abc.MetaPathFinder):
    """Import hook installed when the library is loaded in a process that has
    not imported torch.  The PyTorch wheel bundles its own HIP runtime; once
    this library's runtime (ROCm's) holds the GPU, a torch imported later
    fails its GPU initialisation with a misleading "No HIP GPUs are
    available" ("PyTorch in the same process";
    tools/dbg_torch_after.py).  The guard turns that into a clear error at
    the ``import torch`` that causes it.  It answers ``find_spec`` with a
    spec whose loader raises, so availability probes
    (``importlib.util.find_spec("torch")``) still see torch as installed and
    only an actual import fails."""

    def find_spec(self, name, path=None, target=None):
        # only a torch the other finders would actually import is guarded: in
        # an environment without torch, probes still report it absent
        if name == "torch" and _lib is not None and importlib.machinery.PathFinder.find_spec(name, path) is not None:
            return importlib.util.spec_from_loader(name, _GuardLoader())
        return None


def _order_runtimes():
    """Keep the two HIP runtimes in a working order.  A process that has
    already imported torch is fine as it is.  PHYLO_WITH_TORCH=1 imports
    torch (loaded, not initialised: ~1.5 s, no GPU work) before the library,
    for a process that will use torch later.  Otherwise nothing is imported
    -- a CLI or Stan-style consumer pays nothing for torch -- and the guard
    makes a later ``import torch`` fail loudly instead of leaving torch
    without a GPU."""
    import sys
    if "torch" in sys.modules:
        return
    if os.environ.get("PHYLO_WITH_TORCH") == "1":
        import torch  # noqa: F401
        return
    if not any(isinstance(f, _TorchAfterEngineGuard) for f in sys.meta_path):
        sys.meta_path.insert(0, _TorchAfterEngineGuard())


def load(path=None):
    """Load (once) and return the library.  Raises ``PhyloHipError`` if the
    HIP library has not been built or does not export every entry point of
    ``include/phylo_hip.h`` -- the product has no CPU fallback and no partial
    binding.  ``PHYLO_HIP_AB=1`` (same-box A/B runs of older variant builds,
    ``PHYLO_HIP_LIB``) binds what the variant exports and prints the missing
    names once."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise PhyloHipError(
            "HIP library %s is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback in phylostan_amd)" % p)
    _order_runtimes()
    lib = ctypes.CDLL(p)
    missing = []
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            missing.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    if missing:
        if os.environ.get("PHYLO_HIP_AB") != "1":
            raise PhyloHipError("%s does not export %s (stale build?)" % (p, ", ".join(missing)))
        import sys
        print("phylostan_amd: A/B variant %s lacks %s" % (p, ", ".join(missing)), file=sys.stderr)
    if path is None:
        _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().phy_last_error().decode(errors="replace")
        raise PhyloHipError("%s failed (code %d): %s" % (what, rc, msg))
