"""Wire format of a partisan peer connection (include/partisan_gpu_sim.h
psim_wire_encode / psim_wire_decode): {packet, 4} frames
around partisan_util:term_to_iolist/1 of the manager's messages (what a
partisan connection writes, peer_service_client:95, :275), so simulated nodes can
talk to real partisan nodes.  Records are the engine's 64-B message records
as 16 uint32 words (dst, src, type | ttl << 8 | nex << 16, seq, a0, a1, a2,
a3, ex[8])."""
import ctypes as C

import numpy as np

from . import _lib


class Names(C.Structure):
    """psim_wire_names: node i = '<prefix><i>@<host>' listening on ip_base + i:port"""
    _fields_ = [("prefix", C.c_char_p), ("host", C.c_char_p), ("ip_base", C.c_uint32), ("port", C.c_uint32)]


def names(prefix="n", host="127.0.0.1", ip_base=(10 << 24), port=9090):
    return Names(prefix.encode(), host.encode(), ip_base, port)


def _api():
    lib = _lib.load()
    enc, dec = lib.psim_wire_encode, lib.psim_wire_decode
    enc.restype = dec.restype = C.c_int
    enc.argtypes = [C.POINTER(C.c_uint32), C.POINTER(Names), C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    dec.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(Names), C.c_uint32, C.POINTER(C.c_uint32),
                    C.POINTER(C.c_size_t)]
    return enc, dec


class WireError(ValueError):
    pass


def encode(rec, nm):
    """One record -> one frame (bytes)."""
    enc, _ = _api()
    r = np.ascontiguousarray(rec, np.uint32)
    assert r.size == 16
    n = C.c_size_t()
    rp = r.ctypes.data_as(C.POINTER(C.c_uint32))
    if enc(rp, C.byref(nm), None, 0, C.byref(n)) != 0:
        raise WireError("record has no wire form")
    buf = C.create_string_buffer(n.value)
    enc(rp, C.byref(nm), buf, n.value, C.byref(n))
    return buf.raw[:n.value]


def decode(data, nm, dst):
    """The first frame of `data` -> (record words, bytes used); None if no
    complete frame yet."""
    _, dec = _api()
    r = np.zeros(16, np.uint32)
    used = C.c_size_t()
    b = C.create_string_buffer(bytes(data), len(data))
    rc = dec(b, len(data), C.byref(nm), dst, r.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(used))
    if rc == -5:                                      # PSIM_ERANGE: incomplete frame
        return None
    if rc != 0:
        raise WireError("not a partisan message frame")
    return r, used.value
