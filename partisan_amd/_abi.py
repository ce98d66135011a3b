"""ctypes mirror of include/partisan_gpu_sim.h (plain data types only).

Shared by the product loader (partisan_amd/_lib.py) and the test drivers.
Field order and widths must match the header exactly; tests/test_abi.py checks
the struct sizes against the compiled library.
"""
import ctypes as C

import numpy as np

PSIM_ABI_VERSION = 12
PSIM_MAP_BIT = 0x80000000
PSIM_NONE = 0xFFFFFFFF
ACTIVE_CAP, PASSIVE_CAP, IDMAP_CAP = 8, 32, 64
PT_MEMBERS_CAP, PT_SET_POOL, PT_OUT_CAP, EXCHANGE_CAP = 8, 64, 128, 8
PT_ROOTS, MSG_SLOTS = 4, 64
CONN_CAP, CONN_DOWN, CONN_CLOSING = 8, 0x80000000, 0x40000000
OVF_NKINDS = 5
NTYPES = 24
SVIEW_CAP = 128
MANAGER_HYPARVIEW, MANAGER_PLUGGABLE, MANAGER_XBOT = 0, 1, 2
STRATEGY_FULL, STRATEGY_SCAMP_V1, STRATEGY_SCAMP_V2 = 0, 1, 2

MSG_TYPES = [
    "JOIN", "FORWARD_JOIN", "NEIGHBOR", "DISCONNECT", "NEIGHBOR_REQUEST",
    "NEIGHBOR_ACCEPTED", "NEIGHBOR_REJECTED", "SHUFFLE", "SHUFFLE_REPLY",
    "PT_BROADCAST", "PT_PRUNE", "PT_IHAVE", "PT_IGNORED_IHAVE", "PT_GRAFT", "", "",
    "XBOT_OPTIMIZATION", "XBOT_OPTIMIZATION_REPLY", "XBOT_REPLACE", "XBOT_REPLACE_REPLY",
    "XBOT_SWITCH", "XBOT_SWITCH_REPLY",
]
PL_MSG_TYPES = ["HELLO", "STATE", "GOSSIP", "FWD_SUB", "PING", "KEEP_SUB", "REMOVE_SUB", "BOOT_REMOVE"]
OMIT_SEND, OMIT_RECEIVE = 0, 1
HV_TYPES = list(range(0, 9))
PT_TYPES = list(range(9, 14))
XBOT_TYPES = list(range(16, 22))

ERRORS = {
    0: "PSIM_OK", -1: "PSIM_EINVAL", -2: "PSIM_ENOMEM", -3: "PSIM_EDEVICE",
    -4: "PSIM_ESTATE", -5: "PSIM_ERANGE", -6: "PSIM_ECOMM", -7: "PSIM_EUNSUPPORTED",
    -8: "PSIM_ECAPACITY",
}


class PsimConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32), ("n_nodes", C.c_uint32), ("seed", C.c_uint64),
        ("max_active_size", C.c_uint32), ("min_active_size", C.c_uint32),
        ("max_passive_size", C.c_uint32), ("arwl", C.c_uint32), ("prwl", C.c_uint32),
        ("k_active", C.c_uint32), ("k_passive", C.c_uint32),
        ("shuffle_period", C.c_uint32), ("promotion_period", C.c_uint32),
        ("random_promotion", C.c_uint32), ("persist_epoch", C.c_uint32),
        ("plumtree", C.c_uint32), ("lazy_tick_period", C.c_uint32),
        ("device", C.c_int32), ("n_shards", C.c_uint32), ("shard_rank", C.c_uint32),
        ("shard_world", C.c_uint32), ("comm_id", C.c_void_p),
        ("max_msgs_per_round", C.c_uint64),
        ("manager", C.c_uint32), ("strategy", C.c_uint32), ("periodic_interval", C.c_uint32),
        ("scamp_c", C.c_uint32), ("fanout", C.c_uint32), ("strict", C.c_uint32),
        ("xbot_period", C.c_uint32), ("reserved1", C.c_uint32),
    ]


class PsimRoundStats(C.Structure):
    _fields_ = [
        ("round", C.c_uint64), ("emitted", C.c_uint64 * NTYPES),
        ("delivered", C.c_uint64 * NTYPES), ("dropped", C.c_uint64),
        ("nodes_up", C.c_uint64), ("nodes_processed", C.c_uint64), ("exits", C.c_uint64),
        ("send_fail", C.c_uint64), ("first_deliveries", C.c_uint64), ("overflow", C.c_uint64),
        ("digest", C.c_uint64), ("state_bytes", C.c_uint64), ("overflow_by", C.c_uint64 * OVF_NKINDS),
        ("omitted", C.c_uint64),
    ]


class PsimNodeView(C.Structure):
    _fields_ = [
        ("up", C.c_uint32), ("epoch", C.c_uint32), ("start_round", C.c_uint32),
        ("conn_n", C.c_uint32), ("rng_ctr", C.c_uint64),
        ("act_n", C.c_uint32), ("pas_n", C.c_uint32),
        ("act", C.c_uint32 * ACTIVE_CAP), ("pas", C.c_uint32 * PASSIVE_CAP),
        ("sent_n", C.c_uint32), ("sent_head", C.c_uint32),
        ("recv_n", C.c_uint32), ("recv_head", C.c_uint32),
        ("sent_peer", C.c_uint32 * IDMAP_CAP), ("sent_id", C.c_uint32 * IDMAP_CAP),
        ("recv_peer", C.c_uint32 * IDMAP_CAP), ("recv_id", C.c_uint32 * IDMAP_CAP),
        ("pt_all_n", C.c_uint32), ("pt_common_n", C.c_uint32),
        ("pt_out_n", C.c_uint32), ("pt_pad", C.c_uint32),
        ("pt_all", C.c_uint32 * PT_MEMBERS_CAP), ("pt_common", C.c_uint32 * PT_MEMBERS_CAP),
        ("pt_root", C.c_uint32 * PT_ROOTS), ("pt_eager_n", C.c_uint32 * PT_ROOTS),
        ("pt_lazy_n", C.c_uint32 * PT_ROOTS),
        ("pt_eager", C.c_uint32 * PT_SET_POOL), ("pt_lazy", C.c_uint32 * PT_SET_POOL),
        ("pt_out_peer", C.c_uint32 * PT_OUT_CAP), ("pt_out_msg", C.c_uint32 * PT_OUT_CAP),
        ("pt_out_round", C.c_uint32 * PT_OUT_CAP),
        ("have", C.c_uint64), ("trk_round", C.c_uint32), ("trk_hop", C.c_uint32),
        ("conn", C.c_uint32 * CONN_CAP),
    ]


class PsimStrategyView(C.Structure):
    _fields_ = [
        ("up", C.c_uint32), ("start_round", C.c_uint32), ("pending", C.c_uint32),
        ("last_ping", C.c_uint32), ("rng_ctr", C.c_uint64),
        ("view_n", C.c_uint32), ("in_n", C.c_uint32),
        ("view", C.c_uint32 * SVIEW_CAP), ("in_view", C.c_uint32 * SVIEW_CAP),
        ("members", C.c_uint32), ("view_slots", C.c_uint32), ("members_hash", C.c_uint64),
    ]


HIST_BINS = 64


class PsimHistograms(C.Structure):
    _fields_ = [
        ("n_up", C.c_uint64),
        ("active_in", C.c_uint64 * HIST_BINS), ("passive_in", C.c_uint64 * HIST_BINS),
        ("active_out", C.c_uint64 * HIST_BINS), ("passive_fill", C.c_uint64 * HIST_BINS),
        ("hop", C.c_uint64 * HIST_BINS),
        ("delivered", C.c_uint64), ("last_round", C.c_uint64),
        ("active_links", C.c_uint64), ("symmetric_links", C.c_uint64),
        ("components", C.c_uint64), ("largest_component", C.c_uint64),
        ("reserved", C.c_uint64 * 6),
    ]


NODE_VIEW_DTYPE = np.dtype(PsimNodeView)
STRATEGY_VIEW_DTYPE = np.dtype(PsimStrategyView)
STATS_DTYPE = np.dtype(PsimRoundStats)

# entry points of the C ABI: name -> (restype, argtypes)
_H = C.c_void_p
_P32 = C.POINTER(C.c_uint32)
SIGNATURES = {
    "default_config": (None, [C.POINTER(PsimConfig)]),
    "create": (C.c_int, [C.POINTER(PsimConfig), C.POINTER(C.c_void_p)]),
    "destroy": (None, [_H]),
    "join": (C.c_int, [_H, _P32, _P32, C.c_size_t]),
    "crash": (C.c_int, [_H, _P32, C.c_size_t]),
    "revive": (C.c_int, [_H, _P32, C.c_size_t]),
    "leave": (C.c_int, [_H, _P32, C.c_size_t]),
    "leave_node": (C.c_int, [_H, _P32, _P32, C.c_size_t]),
    "set_partition": (C.c_int, [_H, C.POINTER(C.c_uint8), C.c_size_t]),
    "clear_partition": (C.c_int, [_H]),
    "set_bucket_table": (C.c_int, [_H, C.POINTER(C.c_uint8), C.c_size_t]),
    "set_phash_table": (C.c_int, [_H, _P32, C.c_size_t]),
    "set_omission": (C.c_int, [_H, C.c_int, _P32, _P32, C.c_size_t, C.c_int]),
    "set_faulted": (C.c_int, [_H, _P32, C.c_size_t, C.c_int]),
    "clear_faults": (C.c_int, [_H]),
    "broadcast": (C.c_int, [_H, C.c_uint32, C.c_uint32]),
    "step": (C.c_int, [_H, C.c_uint32, C.POINTER(PsimRoundStats)]),
    "get_nodes": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.POINTER(PsimNodeView)]),
    "get_round": (C.c_int, [_H, C.POINTER(C.c_uint64)]),
    "get_strategy_nodes": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.POINTER(PsimStrategyView)]),
    "get_member_bits": (C.c_int, [_H, C.c_uint32, _P32, C.c_size_t]),
    "get_delivery": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint8), _P32, _P32]),
    "get_histograms": (C.c_int, [_H, C.POINTER(PsimHistograms)]),
    "get_msg_slots": (C.c_int, [_H, _P32, _P32, C.c_size_t]),
    "xbot_latency": (C.c_uint32, [C.c_uint64, C.c_uint32, C.c_uint32]),
}
# symbols only the GPU library exports
GPU_ONLY = {
    "strerror": (C.c_char_p, [C.c_int]),
    "abi_version": (C.c_int, []),
    "kernel_times": (C.c_int, [_H, C.POINTER(C.c_char_p), C.POINTER(C.c_double),
                               C.POINTER(C.c_uint64), C.c_int]),
    "comm_id_size": (C.c_int, []),
    "get_comm_id": (C.c_int, [C.c_void_p, C.c_size_t]),
    "loopback_comm_id": (C.c_int, [C.c_void_p, C.c_size_t]),
    "snapshot": (C.c_int, [_H, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "restore": (C.c_int, [_H, C.c_void_p, C.c_size_t]),
    "get_exchange_stats": (C.c_int, [_H, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "debug_kernel_counts": (C.c_int, [_H, C.POINTER(C.c_uint64), C.c_int]),
}


def bind(lib, prefix, names):
    """Attach restype/argtypes for `prefix + name` and return {name: fn}."""
    out = {}
    for name, (res, args) in names.items():
        fn = getattr(lib, prefix + name)
        fn.restype = res
        fn.argtypes = args
        out[name] = fn
    return out


def u32p(a):
    return a.ctypes.data_as(_P32)
