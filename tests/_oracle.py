"""Test-only loader for the CPU oracle (oracle/liborc.so).  The oracle is the
checker, never the product: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use this module."""
import ctypes as C
import os
import subprocess

from partisan_amd import _abi
from partisan_amd.sim import _Driver

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORC_DIR = os.path.join(ROOT, "oracle")
ORC_PATH = os.path.join(ORC_DIR, "liborc.so")

_lib = None


def load():
    global _lib
    if _lib is None:
        src = os.path.join(ORC_DIR, "psim_oracle.c")
        if not os.path.exists(ORC_PATH) or os.path.getmtime(ORC_PATH) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", ORC_DIR])
        _lib = C.CDLL(ORC_PATH)
        _lib.orc_get_inbox.restype = C.c_int
        _lib.orc_get_inbox.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t,
                                       C.POINTER(C.c_size_t)]
        _lib.orc_philox.restype = None
        _lib.orc_philox.argtypes = [C.c_uint32] * 6 + [C.POINTER(C.c_uint32)]
        _lib.orc_bucket16.restype = C.c_uint32
        _lib.orc_bucket16.argtypes = [C.c_uint32]
    return _lib


class Oracle(_Driver):
    def __init__(self, cfg):
        lib = load()
        super().__init__(_abi.bind(lib, "orc_", _abi.SIGNATURES), cfg)
        self._lib = lib

    def inbox(self):
        import numpy as np

        n = C.c_size_t()
        self._lib.orc_get_inbox(self._h, None, 0, C.byref(n))
        out = np.zeros((n.value, 16), np.uint32)
        self._lib.orc_get_inbox(self._h, out.ctypes.data, n.value, C.byref(n))
        return out
