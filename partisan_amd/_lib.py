"""Loader for the in-tree HIP library.  No fallback: a missing or stale
library is an error, so a GPU run can never silently use another path."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# PSIM_LIB=stamps selects the diagnostic build (profiles/stamps.py); it is the
# same engine with per-phase s_memtime stamps compiled into k_consume
_VARIANT = os.environ.get("PSIM_LIB", "")
LIB_PATH = os.path.join(HERE, "csrc", "libpartisan_gpu_sim%s.so" % ("_" + _VARIANT if _VARIANT else ""))

_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make -C partisan_amd/csrc` "
                "or __graft_entry__.build()")
        _lib = ctypes.CDLL(LIB_PATH)
        from ._abi import PSIM_ABI_VERSION
        if _lib.psim_abi_version() != PSIM_ABI_VERSION:
            raise ImportError("libpartisan_gpu_sim.so ABI version mismatch: rebuild it")
    return _lib
