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
        _lib.orc_round_emit.restype = C.c_int
        _lib.orc_round_emit.argtypes = [C.c_void_p, C.c_void_p]
        _lib.orc_get_outbox.restype = C.c_int
        _lib.orc_get_outbox.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        _lib.orc_round_absorb.restype = C.c_int
        _lib.orc_round_absorb.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
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


class ShardedOracle(Oracle):
    """One rank of the sharded round protocol over a
    torch.distributed process group: emit -> exchange by owner shard ->
    absorb.  Stats of step() are summed over ranks; nodes() covers only the
    owned range."""

    def __init__(self, cfg, group=None):
        import torch.distributed as dist

        self._dist = dist
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._group = group
        cfg.shard_world, cfg.shard_rank = self.world, self.rank
        super().__init__(cfg)
        per = (cfg.n_nodes + self.world - 1) // self.world
        self.lo, self.hi = self.rank * per, min(cfg.n_nodes, (self.rank + 1) * per)
        self.per = per

    def step(self, n_rounds=1):
        import numpy as np
        import torch

        from partisan_amd import _abi

        out = np.zeros(n_rounds, _abi.STATS_DTYPE)
        for i in range(n_rounds):
            st = np.zeros(1, _abi.STATS_DTYPE)
            rc = self._lib.orc_round_emit(self._h, st.ctypes.data)
            assert rc == 0
            n = C.c_size_t()
            self._lib.orc_get_outbox(self._h, None, 0, C.byref(n))
            box = np.zeros((n.value, 16), np.uint32)
            self._lib.orc_get_outbox(self._h, box.ctypes.data, n.value, C.byref(n))
            owner = box[:, 0] // self.per
            parts = [box[owner == g] for g in range(self.world)]   # keeps (src, seq) order
            gathered = [None] * self.world
            self._dist.all_gather_object(gathered, parts, group=self._group)
            mine = np.concatenate([gathered[g][self.rank] for g in range(self.world)]
                                  ).astype(np.uint32).reshape(-1, 16)
            mine = np.ascontiguousarray(mine)
            rc = self._lib.orc_round_absorb(self._h, mine.ctypes.data, mine.shape[0])
            assert rc == 0
            flat = st.view(np.uint64).astype(np.int64)
            t = torch.from_numpy(flat.copy())
            self._dist.all_reduce(t, group=self._group)
            summed = t.numpy().astype(np.uint64)
            summed[0] = st.view(np.uint64)[0]           # the round number is not summed
            out[i] = summed.view(_abi.STATS_DTYPE)[0]
        return out
