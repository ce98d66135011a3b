"""Host-side driver over the C ABI (include/partisan_gpu_sim.h).

`Simulator` is the product entry point: it loads only the HIP library
(libpartisan_gpu_sim.so) and raises if it is missing.  `_Driver` holds the
backend-independent logic so the tests can drive the CPU oracle through the
same code (tests/_oracle.py).
"""
import ctypes as C

import numpy as np

from . import _abi
from .workloads import NONE


class SimError(RuntimeError):
    pass


def default_config(**kw):
    cfg = _abi.PsimConfig()
    cfg.abi_version = _abi.PSIM_ABI_VERSION
    cfg.n_nodes = 32
    cfg.seed = 1
    # partisan_config.erl:102-145 defaults
    cfg.max_active_size, cfg.min_active_size, cfg.max_passive_size = 6, 3, 30
    cfg.arwl, cfg.prwl, cfg.k_active, cfg.k_passive = 5, 30, 3, 4
    cfg.shuffle_period, cfg.promotion_period, cfg.random_promotion = 10, 5, 1
    cfg.persist_epoch, cfg.plumtree, cfg.lazy_tick_period = 0, 1, 1
    cfg.device, cfg.n_shards, cfg.shard_rank, cfg.shard_world = -1, 1, 0, 1
    cfg.comm_id = None
    cfg.max_msgs_per_round = 0
    # pluggable manager (partisan_config.erl:129-130, partisan.hrl:31)
    cfg.manager, cfg.strategy = _abi.MANAGER_HYPARVIEW, _abi.STRATEGY_FULL
    cfg.periodic_interval, cfg.scamp_c, cfg.fanout = 10, 5, 0
    # X-BOT: xbot_interval, 5000 + uniform(60000) ms (partisan_config.erl:100) -> its mean
    cfg.xbot_period = 35
    for k, v in kw.items():
        if not hasattr(cfg, k):
            raise KeyError(k)
        setattr(cfg, k, v)
    return cfg


class _Driver:
    """Backend-independent host logic: event batching, stats decoding."""

    def __init__(self, api, cfg, errname=None):
        self._api = api
        self._errname = errname
        self.cfg = cfg
        self.n = cfg.n_nodes
        h = C.c_void_p()
        self._check(api["create"](C.byref(cfg), C.byref(h)), "create")
        self._h = h

    def _check(self, rc, what):
        if rc != 0:
            msg = _abi.ERRORS.get(rc, str(rc))
            if self._errname is not None:
                msg = self._errname(rc).decode()
            raise SimError(f"{what}: {msg}")

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._api["destroy"](self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- events (applied at the start of the next round)
    def join(self, nodes, contacts):
        nodes = np.ascontiguousarray(nodes, np.uint32)
        contacts = np.ascontiguousarray(contacts, np.uint32)
        assert nodes.shape == contacts.shape
        self._check(self._api["join"](self._h, _abi.u32p(nodes), _abi.u32p(contacts), nodes.size),
                    "join")

    def crash(self, nodes):
        nodes = np.ascontiguousarray(nodes, np.uint32)
        self._check(self._api["crash"](self._h, _abi.u32p(nodes), nodes.size), "crash")

    def revive(self, nodes):
        """Restart nodes without a join (init/1 state, reached by others)."""
        nodes = np.ascontiguousarray(nodes, np.uint32)
        self._check(self._api["revive"](self._h, _abi.u32p(nodes), nodes.size), "revive")

    def leave(self, nodes):
        """leave/0 at each node (pluggable manager; raises on HyParView, whose
        leave answers `error`): the manager stops before its leave messages
        go out, so the node goes down as in crash()."""
        nodes = np.ascontiguousarray(nodes, np.uint32)
        self._check(self._api["leave"](self._h, _abi.u32p(nodes), nodes.size), "leave")

    def leave_node(self, actors, targets):
        """leave/1: actors[i] removes targets[i] (SCAMP v1 / v2 handles)."""
        a = np.ascontiguousarray(actors, np.uint32)
        t = np.ascontiguousarray(targets, np.uint32)
        if a.size != t.size:
            raise ValueError("actors and targets differ in length")
        self._check(self._api["leave_node"](self._h, _abi.u32p(a), _abi.u32p(t), a.size), "leave_node")

    def set_partition(self, group):
        g = np.ascontiguousarray(group, np.uint8)
        self._check(self._api["set_partition"](
            self._h, g.ctypes.data_as(C.POINTER(C.c_uint8)), g.size), "set_partition")

    def clear_partition(self):
        self._check(self._api["clear_partition"](self._h), "clear_partition")

    def set_bucket_table(self, buckets):
        """The sets v1 bucket (erlang:phash(NodeSpec, 16) - 1, 0..15) of every
        node: the view order of SURVEY App. A Q1.  Before the first round;
        None restores the built-in stand-in."""
        if buckets is None:
            self._check(self._api["set_bucket_table"](self._h, None, 0), "set_bucket_table")
            return
        b = np.ascontiguousarray(buckets, np.uint8)
        self._check(self._api["set_bucket_table"](
            self._h, b.ctypes.data_as(C.POINTER(C.c_uint8)), b.size), "set_bucket_table")

    def set_phash_table(self, phash):
        """erlang:phash(NodeSpec, 2^32) - 1 of every node (uint32): the sets
        v1 slots of every set the handle keeps -- 16 buckets for HyParView
        views, the linear hash's wider tables for SCAMP v1 memberships past
        80 ids.  Before the first round; None restores
        the built-in stand-in."""
        if phash is None:
            self._check(self._api["set_phash_table"](self._h, None, 0), "set_phash_table")
            return
        p = np.ascontiguousarray(phash, np.uint32)
        self._check(self._api["set_phash_table"](self._h, _abi.u32p(p), p.size), "set_phash_table")

    # ---- omission faults of the pluggable manager's interposition layer
    # (add_interposition_fun/2, pluggable:297-326; the crash-fault model's
    # begin/end_send_omission, begin/end_receive_omission, begin/end_omission,
    # resolve_all_faults_with_heal: prop_partisan_crash_fault_model:93-229)
    def _omission(self, kind, src, dst, on):
        s = np.ascontiguousarray(np.atleast_1d(src), np.uint32)
        d = np.ascontiguousarray(np.atleast_1d(dst), np.uint32)
        if s.size != d.size:
            raise ValueError("src and dst differ in length")
        self._check(self._api["set_omission"](self._h, kind, _abi.u32p(s), _abi.u32p(d), s.size, int(on)),
                    "set_omission")

    def begin_send_omission(self, src, dst):
        """Messages src forwards to dst are dropped at src (never sent)."""
        self._omission(_abi.OMIT_SEND, src, dst, True)

    def end_send_omission(self, src, dst):
        self._omission(_abi.OMIT_SEND, src, dst, False)

    def begin_receive_omission(self, src, dst):
        """Messages dst receives from src are dropped at dst (never handled)."""
        self._omission(_abi.OMIT_RECEIVE, src, dst, True)

    def end_receive_omission(self, src, dst):
        self._omission(_abi.OMIT_RECEIVE, src, dst, False)

    def begin_omission(self, nodes):
        """General omission: every strategy message the nodes send or receive."""
        n = np.ascontiguousarray(np.atleast_1d(nodes), np.uint32)
        self._check(self._api["set_faulted"](self._h, _abi.u32p(n), n.size, 1), "set_faulted")

    def end_omission(self, nodes):
        n = np.ascontiguousarray(np.atleast_1d(nodes), np.uint32)
        self._check(self._api["set_faulted"](self._h, _abi.u32p(n), n.size, 0), "set_faulted")

    def resolve_all_faults(self):
        self._check(self._api["clear_faults"](self._h), "clear_faults")

    def broadcast(self, root, msg_id):
        self._check(self._api["broadcast"](self._h, root, msg_id), "broadcast")

    # ---- execution
    def step(self, n_rounds=1):
        st = np.zeros(n_rounds, _abi.STATS_DTYPE)
        self._check(self._api["step"](self._h, n_rounds,
                                      st.ctypes.data_as(C.POINTER(_abi.PsimRoundStats))), "step")
        return st

    @property
    def round(self):
        r = C.c_uint64()
        self._check(self._api["get_round"](self._h, C.byref(r)), "get_round")
        return r.value

    def nodes(self, first=0, count=None):
        if count is None:
            count = self.n - first
        out = np.zeros(count, _abi.NODE_VIEW_DTYPE)
        self._check(self._api["get_nodes"](self._h, first, count,
                                           out.ctypes.data_as(C.POINTER(_abi.PsimNodeView))),
                    "get_nodes")
        return out

    def delivery(self, first=0, count=None):
        """Tracked broadcast per node: (have, first-delivery round, hop)."""
        if count is None:
            count = self.n - first
        have = np.zeros(count, np.uint8)
        rnd = np.zeros(count, np.uint32)
        hop = np.zeros(count, np.uint32)
        self._check(self._api["get_delivery"](self._h, first, count,
                                              have.ctypes.data_as(C.POINTER(C.c_uint8)),
                                              _abi.u32p(rnd), _abi.u32p(hop)), "get_delivery")
        return have, rnd, hop

    def msg_slots(self):
        """The live Plumtree message slots (psim_get_msg_slots): per slot k the
        message id owning it (NONE = free) and its root identity."""
        ids = np.zeros(_abi.MSG_SLOTS, np.uint32)
        roots = np.zeros(_abi.MSG_SLOTS, np.uint32)
        self._check(self._api["get_msg_slots"](self._h, _abi.u32p(ids), _abi.u32p(roots), ids.size),
                    "get_msg_slots")
        return ids, roots

    def histograms(self):
        """Overlay statistics (psim_histograms) as a dict of ints / arrays."""
        h = _abi.PsimHistograms()
        self._check(self._api["get_histograms"](self._h, C.byref(h)), "get_histograms")
        out = {}
        for name, _ in _abi.PsimHistograms._fields_:
            if name == "reserved":
                continue
            v = getattr(h, name)
            out[name] = np.array(v[:], np.uint64) if hasattr(v, "__len__") else int(v)
        return out

    def run_schedule(self, schedule, until_round, extra=None):
        """Apply [(round, ids, contacts)] join events and step until `until_round`.
        `extra(round)` may inject further events before each round."""
        ev = {}
        for r, ids, contacts in schedule:
            ev.setdefault(r, []).append((ids, contacts))
        stats = []
        while self.round < until_round:
            r = self.round
            for ids, contacts in ev.get(r, []):
                self.join(ids, contacts)
            if extra is not None:
                extra(r)
            stats.append(self.step(1))
        return np.concatenate(stats) if stats else np.zeros(0, _abi.STATS_DTYPE)

    # ---- pluggable manager state (get_local_state/0, members/0)
    def strategy_nodes(self, first=0, count=None):
        if count is None:
            count = self.n - first
        out = np.zeros(count, _abi.STRATEGY_VIEW_DTYPE)
        self._check(self._api["get_strategy_nodes"](
            self._h, first, count, out.ctypes.data_as(C.POINTER(_abi.PsimStrategyView))),
            "get_strategy_nodes")
        return out

    def member_bits(self, node):
        w = np.zeros((self.n + 31) // 32, np.uint32)
        self._check(self._api["get_member_bits"](self._h, node, _abi.u32p(w), w.size),
                    "get_member_bits")
        return w

    def members(self, node):
        """membership_list/1 of a node: full -> ids of query(ORSet) in id order;
        scamp -> the view in its list order"""
        if self.cfg.strategy == _abi.STRATEGY_FULL:
            w = self.member_bits(node)
            return [int(i) for i in np.nonzero(np.unpackbits(w.view(np.uint8), bitorder="little"))[0]]
        v = self.strategy_nodes(node, 1)[0]
        return [int(x) for x in v["view"][: v["view_n"]]]

    # ---- reference-style debug getters (hyparview:261-281)
    def active(self, node):
        v = self.nodes(node, 1)[0]
        return [int(x) for x in v["act"][: v["act_n"]]]

    def passive(self, node):
        v = self.nodes(node, 1)[0]
        return [int(x) for x in v["pas"][: v["pas_n"]]]


def comm_id():
    """A fresh RCCL unique id (rank 0 creates it and shares the bytes)."""
    from . import _lib

    lib = _lib.load()
    extra = _abi.bind(lib, "psim_", _abi.GPU_ONLY)
    n = extra["comm_id_size"]()
    buf = C.create_string_buffer(n)
    rc = extra["get_comm_id"](buf, n)
    if rc != 0:
        raise SimError(f"get_comm_id: {extra['strerror'](rc).decode()}")
    return buf.raw


def loopback_comm_id():
    """TEST VEHICLE: the id of a new loopback world (psim_loopback_comm_id):
    ranks as threads of this process on one device, in place of RCCL."""
    from . import _lib

    lib = _lib.load()
    extra = _abi.bind(lib, "psim_", _abi.GPU_ONLY)
    n = extra["comm_id_size"]()
    buf = C.create_string_buffer(n)
    rc = extra["loopback_comm_id"](buf, n)
    if rc != 0:
        raise SimError(f"loopback_comm_id: {extra['strerror'](rc).decode()}")
    return buf.raw


class Simulator(_Driver):
    """MI355X simulator handle (HIP library; fails loudly without it).

    Multi-GPU: one process per GPU, all with the same global n_nodes and
    `shard_world`, each with its `shard_rank` and the same `comm` bytes from
    comm_id() on rank 0; every rank then issues the same event calls."""

    def __init__(self, cfg=None, comm=None, **kw):
        from . import _lib

        lib = _lib.load()
        api = _abi.bind(lib, "psim_", _abi.SIGNATURES)
        extra = _abi.bind(lib, "psim_", _abi.GPU_ONLY)
        self._extra = extra
        if cfg is None:
            cfg = default_config(**kw)
        if comm is not None:
            self._comm_buf = C.create_string_buffer(bytes(comm), len(comm))
            cfg.comm_id = C.cast(self._comm_buf, C.c_void_p)
        super().__init__(api, cfg, errname=extra["strerror"])

    def snapshot(self):
        """The whole simulation state as bytes (psim_snapshot)."""
        need = C.c_size_t()
        self._check(self._extra["snapshot"](self._h, None, 0, C.byref(need)), "snapshot")
        buf = C.create_string_buffer(need.value)
        self._check(self._extra["snapshot"](self._h, buf, need.value, C.byref(need)), "snapshot")
        return buf.raw[:need.value]

    def restore(self, data):
        """Load a snapshot into this handle (same config)."""
        buf = C.create_string_buffer(bytes(data), len(data))
        self._check(self._extra["restore"](self._h, buf, len(data)), "restore")

    def exchange_stats(self):
        """(records, wire bytes) this process's shards sent to other shards
        since creation (psim_get_exchange_stats)."""
        r, b = C.c_uint64(), C.c_uint64()
        self._check(self._extra["get_exchange_stats"](self._h, C.byref(r), C.byref(b)), "get_exchange_stats")
        return r.value, b.value

    # (k_node_prep: the quiet lazy ticks it counts without running the node)
    KERNELS = ("k_relay", "k_shuf", "k_lite_half", "k_consume", "k_ptl", "k_pt", "k_node_prep")

    def kernel_counts(self):
        """{kernel: (nodes processed, delivered, emitted)} of the last round,
        per node-round kernel (psim_debug_kernel_counts); {} under the
        pluggable manager."""
        out = (C.c_uint64 * 28)()
        k = self._extra["debug_kernel_counts"](self._h, out, 28)
        self._check(min(k, 0), "debug_kernel_counts")
        return {self.KERNELS[i]: (out[4 * i], out[4 * i + 1], out[4 * i + 2]) for i in range(k)}

    def kernel_times(self):
        cap = 64
        names = (C.c_char_p * cap)()
        ms = (C.c_double * cap)()
        launches = (C.c_uint64 * cap)()
        k = self._extra["kernel_times"](self._h, names, ms, launches, cap)
        return {names[i].decode(): (ms[i], launches[i]) for i in range(k)}


__all__ = ["Simulator", "SimError", "default_config", "comm_id", "NONE"]
