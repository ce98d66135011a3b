"""GPU parity: the HIP engine against the CPU oracle, bit for bit, through
the C ABI.  Every round's statistics (per-type message counts and a digest of
every emitted message including its per-sender sequence number) and every
node's full state after the run must be identical."""
import numpy as np
import pytest

import _scenarios as S
from _oracle import Oracle

pytestmark = pytest.mark.gpu


def _gpu(cfg):
    from partisan_amd import Simulator
    return Simulator(cfg)


def _both(fn, *a, **kw):
    g = fn(_gpu, *a, **kw)
    o = fn(Oracle, *a, **kw)
    return g, o


def test_gpu_loads_native_library():
    from partisan_amd import _abi, _lib
    lib = _lib.load()
    assert lib.psim_abi_version() == _abi.PSIM_ABI_VERSION


def test_config_a_parity():
    (gs, gst), (os_, ost) = _both(S.config_a)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_doubling_parity(seed):
    (gs, gst), (os_, ost) = _both(S.doubling, 1024, seed, 60, bcast_period=10, bcast_first=25)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_churn_partition_parity():
    (gs, gst), (os_, ost) = _both(S.churn_partition, n=2048)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


@pytest.mark.parametrize("kw", [dict(), dict(period=1, snap_at=(60, 79))], ids=["tail", "at_cap"])
def test_outstanding_tail_parity(kw):
    """Outstanding tables past one 64-lane register (up to PSIM_PT_OUT_CAP
    128; tests/test_out_tail.py shows the oracle fills them): adds, acks
    and lazy ticks over the extension row's tail, GPU == oracle, the tables
    compared while at their largest.  (neighbors_down/2's filter over a
    tail, out_drop_peer, is not reached: the entries are lazy-set peers,
    node_spec identities, and the filter drops bare ids -- DESIGN.md 2's
    leak.)"""
    (gs, gst, gsn), (os_, ost, osn) = _both(S.out_tail, **kw)
    S.compare_stats(gst, ost)
    for r in osn:
        S.compare_nodes(gsn[r], osn[r])
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_outstanding_pool_growth(monkeypatch):
    """The outstanding tables' extension pool starting at 8 rows
    (PSIM_OUTX_ROWS): grow_outx doubles it at round boundaries as nodes take
    rows, with no overflow and GPU == oracle through the tables' largest
    (a snapshot of the grown pool restores into a fresh handle)"""
    monkeypatch.setenv("PSIM_OUTX_ROWS", "8")
    gs, gst, gsn = S.out_tail(_gpu)
    os_, ost, osn = S.out_tail(Oracle)
    S.compare_stats(gst, ost)
    for r in osn:
        S.compare_nodes(gsn[r], osn[r])
    assert int(gst["overflow"].sum()) == 0
    assert int((osn[79]["pt_out_n"] > 16).sum()) > 8      # more rows than the pool started with
    snap = gs.snapshot()
    monkeypatch.setenv("PSIM_OUTX_ROWS", "8")
    from partisan_amd.sim import default_config
    fresh = _gpu(default_config(n_nodes=512, seed=3))
    fresh.restore(snap)
    S.compare_nodes(fresh.nodes(), os_.nodes())


def test_kernel_counts_sum_to_the_round():
    """psim_debug_kernel_counts: the node-round kernels' own nodes processed,
    deliveries and emissions add up to the round's stats (every one of them
    is counted by exactly one kernel), round after round of a churn +
    partition run with broadcasts"""
    from partisan_amd.sim import default_config
    from partisan_amd import workloads as W
    n = 2048
    sim = _gpu(default_config(n_nodes=n, seed=5))
    sim.run_schedule(W.doubling_join(n, 5), 40)
    for r in range(40):
        if r % 10 == 0:
            sim.broadcast(0, r)
        if r == 20:
            sim.crash(np.arange(100, 140, dtype=np.uint32))
        st = sim.step(1)
        kc = sim.kernel_counts()
        assert set(kc) == set(sim.KERNELS)
        assert sum(v[0] for v in kc.values()) == int(st["nodes_processed"][0])
        assert sum(v[1] for v in kc.values()) == int(st["delivered"][0].sum())
        assert sum(v[2] for v in kc.values()) == int(st["emitted"][0].sum())


def test_lingering_connections_parity():
    """connections beyond the active view -- shuffle
    terminals' Senders, rejected and pending neighbor requests, a joiner's
    contact -- in the connection table, EXIT at every holder, Plumtree sends
    over them: the crash of the most-held lingering peers, GPU == oracle."""
    (gs, gst, gv), (os_, ost, ov) = _both(S.lingering_exits)
    assert gv == ov and ov
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    assert int((os_.nodes()["conn_n"] > 0).sum()) > 0


def test_e_miniature_parity():
    """Config E in miniature (bench.py's sharding-check schedule) at 2^14
    nodes: churn, restarts, a partition and broadcasts, GPU == oracle."""
    (gs, gst), (os_, ost) = _both(S.e_miniature)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_crash_parity():
    (gs, gst, _), (os_, ost, _) = _both(S.crash_only)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_crash_revive_parity():
    (gs, gst, _), (os_, ost, _) = _both(S.crash_revive)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


@pytest.mark.parametrize("n", [512, 1 << 16])
def test_star_hotspot_parity(n):
    """every node joins node 0 in one round; at 2^16 the JOINs overflow
    their route bucket's fixed region (k_bucket_fill: 1.5x the bucket's
    share of the route capacity) and that round goes through the four-pass
    route again"""
    (gs, gst), (os_, ost) = _both(S.star, n=n)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_variants_parity():
    kw = dict(max_active_size=8, max_passive_size=20, arwl=6, prwl=6, persist_epoch=1)
    (gs, gst), (os_, ost) = _both(S.churn_partition, n=1024, seed=13, rounds=110, **kw)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


@pytest.mark.parametrize("seed", [3, 4])
def test_forward_join_revert_parity(seed):
    """hv:896-897: a FORWARD_JOIN whose TTL == prwl inserted the joiner into
    the passive view, found no forward target and could not reach the
    joiner returns State0 -- the insert is undone, its draw stays consumed.
    Variant config (arwl = prwl = 6) with joiners crashing mid-walk."""
    (gs, gst), (os_, ost) = _both(S.joiner_crash, seed=seed, **S.VARIANT)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_64k_parity():
    """2^16 nodes, 60 rounds + a broadcast: still cheap for the oracle (~5 s)."""
    def run(make):
        sim, st = S.doubling(make, 1 << 16, 21, 60)
        sim.broadcast(0, 5)
        return sim, np.concatenate([st, sim.step(40)])
    (gs, gst), (os_, ost) = _both(run)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_config_c_1m_parity():
    """Config C at its full size (BASELINE.json configs[2]): 2^20 nodes, the
    bench's doubling bootstrap, 20 settle rounds, then a broadcast from node 0
    and 20 rounds more -- every round's statistics and digest and every
    node's final state bit-identical to the oracle (~40 s of oracle time)."""
    def run(make):
        sim, st = S.doubling(make, 1 << 20, 1, 41)
        sim.broadcast(0, 0)
        return sim, np.concatenate([st, sim.step(20)])
    (gs, gst), (os_, ost) = _both(run)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    assert int(gst["first_deliveries"].sum()) > 0


def test_large_properties():
    """2^18 nodes: size-independent properties (the oracle is not run):
    view bounds, broadcast reliability, message conservation (every message
    emitted in round r is delivered or dropped in round r+1)."""
    gs, st = S.doubling(_gpu, 1 << 18, 21, 60)
    gs.broadcast(0, 5)
    st2 = gs.step(40)
    v = gs.nodes()
    assert (v["act_n"] <= 6).all() and (v["pas_n"] <= 30).all()
    assert ((v["have"] >> 5) & 1).mean() > 0.999
    allst = np.concatenate([st, st2])
    em = allst["emitted"].sum(1)[:-1]
    dl = allst["delivered"].sum(1)[1:] + allst["dropped"][1:]
    assert np.array_equal(em, dl)
    assert allst["overflow"].sum() == 0
    assert int(allst["first_deliveries"].sum()) == int(((v["have"] >> 5) & 1).sum()) - 1


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_shard_count_invariance(shards):
    """Node-range sharding (virtual shards on one GPU, exchanged by device
    copies through the same partition/exchange/merge path the RCCL ranks
    use) is bit-identical to the unsharded run and to the oracle."""
    def gpu_sharded(cfg):
        cfg.n_shards = shards
        return _gpu(cfg)
    gs, gst = S.churn_partition(gpu_sharded, n=2048)
    os_, ost = S.churn_partition(Oracle, n=2048)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    # the wire format: 32 B a record, 32 more for one with exchange ids
    # (SHUFFLE / SHUFFLE_REPLY) -- fewer bytes than the 64-B records, and
    # at least every record's head
    xr, xb = gs.exchange_stats()
    assert xr > 0 and 32 * xr < xb < 64 * xr


@pytest.mark.parametrize("shards", [2, 4])
def test_shard_invariance_multistep_blocks(shards, monkeypatch):
    """The route and the owner partition with few blocks (PSIM_ROUTE_BLOCKS=3),
    so every block runs several consecutive source steps, as at >= 2^19
    nodes per shard: still bit-identical to the oracle (a grid-stride step
    order broke the partition's (src, seq) order there)."""
    monkeypatch.setenv("PSIM_ROUTE_BLOCKS", "3")

    def gpu_sharded(cfg):
        cfg.n_shards = shards
        return _gpu(cfg)
    gs, gst = S.churn_partition(gpu_sharded, n=4096)
    os_, ost = S.churn_partition(Oracle, n=4096)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_shard_invariance_64k():
    def run(make):
        sim, st = S.doubling(make, 1 << 16, 21, 60)
        sim.broadcast(0, 5)
        return sim, np.concatenate([st, sim.step(30)])

    def g1(cfg):
        return _gpu(cfg)

    def g4(cfg):
        cfg.n_shards = 4
        return _gpu(cfg)
    (a, ast), (b, bst) = run(g1), run(g4)
    S.compare_stats(ast, bst)
    S.compare_nodes(a.nodes(), b.nodes())


# ---- pluggable manager + membership strategies
@pytest.mark.parametrize("strategy,n,fanout", [(0, 16, 0), (0, 2048, 5), (1, 2048, 0), (2, 2048, 0)])
def test_strategy_parity(strategy, n, fanout):
    (gs, gst), (os_, ost) = _both(S.pl_doubling, n, 11, 100, strategy=strategy, fanout=fanout,
                                  crash_at=40, part_at=60)
    S.compare_stats(gst, ost)
    S.compare_strategy(gs, os_, full_bits=[0, 1, n // 2, n - 1] if strategy == 0 else None)


@pytest.mark.parametrize("strategy", [0, 1, 2])
def test_strategy_leave_parity(strategy):
    """psim_leave (leave/0: the manager stops before its leave messages go
    out) at round 40 for 10% of the nodes, then a partition: bit-identical
    to the oracle."""
    kw = dict(strategy=strategy, fanout=5 if strategy == 0 else 0, crash_at=40, part_at=60, leave=True)
    (gs, gst), (os_, ost) = _both(S.pl_doubling, 1024, 11, 90, **kw)
    S.compare_stats(gst, ost)
    S.compare_strategy(gs, os_, full_bits=[0, 1, 512, 1023] if strategy == 0 else None)


@pytest.mark.parametrize("strategy", [1, 2])
def test_strategy_remote_leave_parity(strategy):
    """psim_leave_node (leave/1, stops mid-round dropping the manager's sends,
    down from the next round) and a partition: bit-identical to the oracle,
    unsharded and over 4 virtual shards."""
    def sharded(cfg):
        cfg.n_shards = 4
        return _gpu(cfg)
    os_, ost, _, _ = S.pl_leave_remote(Oracle, 2048, 7, 90, strategy=strategy, part_at=60)
    for make in (_gpu, sharded):
        gs, gst, _, _ = S.pl_leave_remote(make, 2048, 7, 90, strategy=strategy, part_at=60)
        S.compare_stats(gst, ost)
        S.compare_strategy(gs, os_)


@pytest.mark.parametrize("strategy,n,fanout", [(0, 32, 0), (0, 2048, 5), (1, 2048, 0), (2, 2048, 0)])
def test_omission_fault_parity(strategy, n, fanout):
    """The crash-fault model's omissions (general, send, receive; partly
    ended, then healed) through the interposition layer: bit-identical to
    the oracle, unsharded and over 4 virtual shards (SCAMP)."""
    def sharded(cfg):
        cfg.n_shards = 4
        return _gpu(cfg)
    os_, ost, _ = S.pl_omission(Oracle, n, 23, 100, strategy, fanout)
    assert ost["omitted"].sum() > 0
    for make in (_gpu, sharded) if strategy else (_gpu,):
        gs, gst, _ = S.pl_omission(make, n, 23, 100, strategy, fanout)
        S.compare_stats(gst, ost)
        S.compare_strategy(gs, os_, full_bits=[0, 1, n // 2, n - 1] if strategy == 0 else None)


@pytest.mark.parametrize("n,fanout", [(32, 0), (2048, 5)])
def test_full_remote_leave_parity(n, fanout):
    """psim_leave_node under the full strategy: ORSet remove rows (tombstones)
    merged with the adds, the two-row gossip payload, a target stopping on a
    merged removal of itself -- bit-identical to the oracle (full-strategy
    handles are single-shard: gossip payloads are shard-local)."""
    kw = dict(strategy=0, fanout=fanout, k=4, part_at=60)
    os_, ost, _, _ = S.pl_leave_remote(Oracle, n, 8, 90, **kw)
    gs, gst, _, _ = S.pl_leave_remote(_gpu, n, 8, 90, **kw)
    S.compare_stats(gst, ost)
    S.compare_strategy(gs, os_, full_bits=[0, 1, n // 2, n - 1])


@pytest.mark.parametrize("strategy", [1, 2])
def test_strategy_shard_invariance(strategy):
    def sharded(cfg):
        cfg.n_shards = 4
        return _gpu(cfg)
    gs, gst = S.pl_doubling(sharded, 4096, 12, 80, strategy=strategy, crash_at=40)
    os_, ost = S.pl_doubling(Oracle, 4096, 12, 80, strategy=strategy, crash_at=40)
    S.compare_stats(gst, ost)
    S.compare_strategy(gs, os_)


def test_strategy_64k_parity():
    (gs, gst), (os_, ost) = _both(S.pl_doubling, 1 << 16, 13, 60, strategy=2)
    S.compare_stats(gst, ost)
    S.compare_strategy(gs, os_)


def test_gpu_matches_committed_oracle_traces():
    """The GPU engine against tests/golden/oracle_traces.json directly (the
    committed per-round digests of the oracle scenarios)."""
    import json
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    import gen_oracle_traces as G
    golden = json.load(open(os.path.join(here, "golden", "oracle_traces.json")))["traces"]
    scen = {
        "config_a": lambda: S.config_a(_gpu),
        "churn_partition_1024": lambda: S.churn_partition(_gpu, n=1024),
        "full_16_fanout0": lambda: S.pl_doubling(_gpu, 16, 11, 80, strategy=0, fanout=0, crash_at=40),
        "full_1024_fanout5": lambda: S.pl_doubling(_gpu, 1024, 11, 80, strategy=0, fanout=5, part_at=50),
        "scamp_v1_1024": lambda: S.pl_doubling(_gpu, 1024, 11, 100, strategy=1, crash_at=40, part_at=60),
        "scamp_v2_1024": lambda: S.pl_doubling(_gpu, 1024, 11, 100, strategy=2, crash_at=40, part_at=60),
        "scamp_v1_leave_1024": lambda: S.pl_leave_remote(_gpu, 1024, 7, 90, strategy=1, part_at=60)[:2],
        "scamp_v2_leave_1024": lambda: S.pl_leave_remote(_gpu, 1024, 7, 90, strategy=2, part_at=60)[:2],
        "full_leave_1024_fanout5": lambda: S.pl_leave_remote(_gpu, 1024, 8, 90, strategy=0, fanout=5, k=4)[:2],
    }
    assert set(scen) == set(G.SCENARIOS)
    for name, run in scen.items():
        _, st = run()
        got = [int(x) for x in st["digest"]]
        assert got == golden[name]["digest"], (name, st["emitted"].sum(1)[:8].tolist(),
                                               st["nodes_processed"][:8].tolist(), got[:4])


def test_route_regrow_parity(monkeypatch):
    """A route capacity of 16 records forces the device-side overflow check,
    the host's regrow and the reroute of the same outbox in most early
    rounds (PSIM_RCAP_INIT, psim_engine.hip); results stay bit-identical."""
    monkeypatch.setenv("PSIM_RCAP_INIT", "16")
    (gs, gst), (os_, ost) = _both(S.doubling, 1024, 4, 40, bcast_period=10, bcast_first=15)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_batch_regrow_parity(monkeypatch):
    """Batched rounds (run_batch, psim_engine.hip) whose outbox and route
    outgrow their buffers mid-batch: with no up-front reservation and a
    route capacity of 16 records the abort word stops batches at k_desc
    (code 1) and at the route (code 2); the host grows the buffer, finishes
    that round and starts the next batch.  Results stay bit-identical."""
    monkeypatch.setenv("PSIM_NO_RESERVE", "1")
    monkeypatch.setenv("PSIM_RCAP_INIT", "16")

    def run(make):
        sim, _ = S.doubling(make, 4096, 9, 30, bcast_period=0, bcast_first=0)
        sim.broadcast(7, 1)
        out = [sim.step(60)]                      # one step call: batches, growth inside
        sim.crash(np.arange(3, 4096, 37, dtype=np.uint32))
        out.append(sim.step(40))
        return sim, out
    (gs, gst), (os_, ost) = run(_gpu), run(Oracle)
    for a, b in zip(gst, ost):
        S.compare_stats(a, b)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_histograms_delivery_parity():
    """psim_get_histograms / psim_get_delivery: the GPU's device kernels
    (in-degree atomics, reverse-link test, label propagation) against the
    oracle's list-style statistics on the same run."""
    def run(make):
        sim, _ = S.doubling(make, 2048, 3, 70, bcast_period=25, bcast_first=30)
        sim.crash(np.arange(5, 2048, 61, dtype=np.uint32))
        sim.step(2)
        return sim
    g, o = run(_gpu), run(Oracle)
    hg, ho = g.histograms(), o.histograms()
    for k in ho:
        assert np.array_equal(np.asarray(hg[k]), np.asarray(ho[k])), k
    for a, b in zip(g.delivery(), o.delivery()):
        assert np.array_equal(a, b)
    assert hg["components"] == 1


def test_duplicate_join_rejected_gpu():
    """The engine refuses a second start of a pending id (EINVAL), as the
    oracle does; the run then matches the oracle."""
    from partisan_amd.sim import default_config

    def run(make):
        sim = make(default_config(n_nodes=64, seed=4))
        with pytest.raises(Exception):
            sim.join(np.array([0, 0], np.uint32), np.array([0xFFFFFFFF, 0xFFFFFFFF], np.uint32))
        sim.join(np.array([0], np.uint32), np.array([0xFFFFFFFF], np.uint32))
        sim.step(1)
        ids = np.arange(1, 64, dtype=np.uint32)
        sim.join(ids, np.zeros(63, np.uint32))
        with pytest.raises(Exception):
            sim.join(ids[5:6], np.zeros(1, np.uint32))
        return sim, sim.step(30)
    (g, gst), (o, ost) = run(_gpu), run(Oracle)
    S.compare_stats(gst, ost)
    S.compare_nodes(g.nodes(), o.nodes())


@pytest.mark.parametrize("shards", [1, 4])
def test_histograms_large_properties(shards):
    """Overlay statistics at 2^22 nodes (the oracle is not run): symmetric
    links <= active links, every histogram sums to the live nodes, the link
    and in-degree totals agree, and a host recount over the node rows
    (active in-degrees, symmetric links, out-degrees) matches.  With 4
    virtual shards the statistics must equal the unsharded ones (the
    gathered-row symmetry / components path of sharded handles)."""
    def make(cfg):
        cfg.n_shards = shards
        return _gpu(cfg)
    n = 1 << 22
    sim, _ = S.doubling(make, n, 7, 40)
    sim.broadcast(0, 3)
    sim.step(30)
    h = sim.histograms()
    up = h["n_up"]
    assert up == n
    for k in ("active_in", "passive_in", "active_out", "passive_fill"):
        assert int(h[k].sum()) == up, k
    assert h["symmetric_links"] <= h["active_links"]
    bins = np.arange(len(h["active_in"]), dtype=np.uint64)
    assert int((h["active_in"] * bins).sum()) == h["active_links"]
    assert int((h["active_out"] * bins).sum()) == h["active_links"]
    assert h["delivered"] == int(h["hop"].sum())
    v = sim.nodes()
    act = v["act"].astype(np.int64)
    k = np.arange(8)[None, :] < v["act_n"][:, None].astype(np.int64)
    me = np.arange(n)[:, None]
    link = k & (act != me)
    src = np.broadcast_to(me, act.shape)[link]
    dst = act[link]
    assert link.sum() == h["active_links"]
    assert np.array_equal(np.bincount(np.minimum(np.bincount(dst, minlength=n), 63), minlength=64),
                          h["active_in"].astype(np.int64))
    fwd = np.unique(src * n + dst)
    rev = np.unique(dst * n + src)
    assert np.intersect1d(fwd, rev, assume_unique=True).size == h["symmetric_links"]
    global _HIST_1
    if shards == 1:
        _HIST_1 = h
    elif "_HIST_1" in globals():
        for kk in _HIST_1:
            assert np.array_equal(np.asarray(h[kk]), np.asarray(_HIST_1[kk])), kk


@pytest.mark.parametrize("roots,rounds,churn", [(4, 200, False), (4, 160, True), (6, 120, False)])
def test_multi_root_parity(roots, rounds, churn):
    """Several Plumtree roots at once (per-root eager / lazy sets in 4 root
    slots, pt:76-84, :599-631; message ids past the 64 message slots): the
    engine equals the oracle, with 4 roots (no overflow), under churn, and
    with 6 roots (full root slots, counted as overflow identically)."""
    (gs, gst, _), (os_, ost, _) = _both(S.multi_root, roots=roots, rounds=rounds, churn=churn)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    if roots <= 4 and not churn:
        assert int(gst["overflow"].sum()) == 0


def test_multi_root_shard_invariance():
    """Four roots over 3 virtual shards: bit-identical to the oracle."""
    def g3(cfg):
        cfg.n_shards = 3
        return _gpu(cfg)
    (gs, gst, _), (os_, ost, _) = S.multi_root(g3, roots=4, rounds=120), S.multi_root(Oracle, roots=4, rounds=120)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_snapshot_restore_continues_identically():
    """psim_snapshot after 60 rounds, restored into a fresh handle: the next
    40 rounds (a broadcast included) are identical to the original's."""
    from partisan_amd import Simulator
    from partisan_amd.sim import default_config
    sim, _ = S.doubling(_gpu, 4096, 2, 60)
    snap = sim.snapshot()
    sim.broadcast(0, 7)
    a = sim.step(40)
    other = Simulator(default_config(n_nodes=4096, seed=2))
    # a short snapshot (its last section cut) is refused before anything
    # changes: the fresh handle still steps as a fresh handle
    from partisan_amd.sim import SimError
    with pytest.raises(SimError):
        other.restore(snap[:-64])
    assert other.round == 0
    other.step(1)
    other.restore(snap)
    assert other.round == 60
    other.broadcast(0, 7)
    b = other.step(40)
    S.compare_stats(a, b)
    S.compare_nodes(sim.nodes(), other.nodes())


def test_failed_step_poisons_until_restore():
    """a round that fails half-way leaves the handle answering PSIM_ESTATE
    until psim_restore puts it back on a round boundary; a snapshot made
    under one view-order table is refused under another (tests/_fail_run.py,
    a child process: the failure hook is read once per process)"""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, PSIM_TEST_FAIL_ROUND="50")
    r = subprocess.run([sys.executable, "-u", os.path.join(here, "_fail_run.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def test_msg_slots_and_strict_gpu():
    """psim_get_msg_slots and cfg.strict on the GPU: six live roots overflow
    the four root slots -- counted identically to the oracle by default, a
    failed step (PSIM_ECAPACITY) with strict = 1."""
    from partisan_amd.sim import SimError
    (gs, gst, _), (os_, ost, _) = _both(S.multi_root, n=512, roots=6, rounds=60)
    S.compare_stats(gst, ost)
    for a, b in zip(gs.msg_slots(), os_.msg_slots()):
        assert np.array_equal(a, b)
    with pytest.raises(SimError, match="overflowed"):
        S.multi_root(_gpu, n=512, roots=6, rounds=60, strict=1)


def test_heartbeat_parity():
    """Every node a root (plumtree_backend's heartbeat, backend:179-200):
    64 nodes beating every 10 rounds overflow the 4 root slots; GPU and
    oracle count the same overflows (strict = 0) and both fail the step with
    strict = 1 (the test above covers the GPU's error)."""
    (gs, gst), (os_, ost) = _both(S.heartbeat)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())
    assert int(ost["overflow_by"][:, 2].sum()) > 0


@pytest.mark.parametrize("name", ["C_survey", "C_doubling"])
def test_bench_schedule_parity(name):
    """bench.py's exact schedules (workloads.BenchSchedule) at the bench's
    2^20 nodes, into the timed window -- for the survey line the driver's
    whole window (--warmup 5, the 20 timed rounds of the broadcast's
    propagation, 5 more), or two broadcasts and a cohort merge round of the
    doubling line --
    against the oracle's committed run of the same schedule
    (tests/golden/gen_bench_fixtures.py): every round's digest and counts,
    and the hash of every node's final view."""
    import hashlib
    import json
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    import gen_bench_fixtures as G
    fx = json.load(open(os.path.join(here, "golden", "bench_fixtures.json")))
    want = fx["fixtures"][name]
    wu = fx["warmup"][name] if isinstance(fx["warmup"], dict) else fx["warmup"]
    st, nodes = G.run(_gpu, name, n=fx["nodes"], seed=fx["seed"], warmup=wu, window=fx["window"][name])
    assert len(st) == want["rounds"]
    for f in G.FIELDS:
        got = st[f].tolist()
        if got != want[f]:
            bad = next(i for i, (a, b) in enumerate(zip(got, want[f])) if a != b)
            raise AssertionError(f"{name}: {f} differs first at round {bad}")
    assert hashlib.sha256(nodes.tobytes()).hexdigest() == want["state_sha256"]


# ---- X-BOT (partisan_hyparview_xbot_peer_service_manager)
@pytest.mark.parametrize("period", [35, 10])
def test_xbot_parity(period):
    """X-BOT's optimization rounds (xbot:586-606, :691-716, :1171-1346) under
    churn and a partition: the discarded-state connects and disconnects,
    the stopped pids' EXITs one round later, the JOIN / FORWARD_JOIN /
    NEIGHBOR_REQUEST variants -- GPU == oracle (period 10: a busier overlay
    whose id-map and connection-table overflows are counted identically)."""
    (gs, gst), (os_, ost) = _both(S.churn_partition, n=2048, manager=2, xbot_period=period)
    assert ost["emitted"][:, 16:22].sum() > 1000
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_xbot_shard_invariance():
    def gpu_sharded(cfg):
        cfg.n_shards = 3
        return _gpu(cfg)
    gs, gst = S.churn_partition(gpu_sharded, n=2048, manager=2, xbot_period=20)
    os_, ost = S.churn_partition(Oracle, n=2048, manager=2, xbot_period=20)
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def test_xbot_64k_parity():
    (gs, gst), (os_, ost) = _both(S.doubling, 1 << 16, 31, 70, bcast_period=10, bcast_first=30,
                                  manager=2, xbot_period=12)
    assert ost["emitted"][:, 16:22].sum() > 10000
    S.compare_stats(gst, ost)
    S.compare_nodes(gs.nodes(), os_.nodes())


def _both_tab(fn, seed, *a, **kw):
    return fn(S.with_buckets(_gpu, seed), *a, **kw), fn(S.with_buckets(Oracle, seed), *a, **kw)


@pytest.mark.parametrize("case", ["config_a", "churn_partition", "doubling_64k", "xbot", "scamp_v1"])
def test_bucket_table_parity(case):
    """App. A Q1: a sets v1 bucket table that is not the built-in stand-in
    (psim_set_bucket_table, what an in-BEAM harness export of
    erlang:phash(NodeSpec, 16) supplies) -- GPU == oracle bit for bit, and
    the views follow the table."""
    if case == "config_a":
        (gs, gst), (os_, ost) = _both_tab(S.config_a, 11)
    elif case == "churn_partition":
        (gs, gst), (os_, ost) = _both_tab(S.churn_partition, 12, n=2048)
    elif case == "doubling_64k":
        def run(make):
            sim, st = S.doubling(make, 1 << 16, 21, 60)
            sim.broadcast(0, 5)
            return sim, np.concatenate([st, sim.step(30)])
        (gs, gst), (os_, ost) = _both_tab(run, 13)
    elif case == "xbot":
        (gs, gst), (os_, ost) = _both_tab(S.xbot_churn, 14, n=1024, rounds=100)
    else:
        (gs, gst), (os_, ost) = _both_tab(S.pl_doubling, 15, 2048, 5, 60, 1, crash_at=30, part_at=40)
        S.compare_stats(gst, ost)
        S.compare_strategy(gs, os_)
        return
    S.compare_stats(gst, ost)
    v = gs.nodes()
    S.compare_nodes(v, os_.nodes())
    tab = S.random_buckets(len(v), {"config_a": 11, "churn_partition": 12, "doubling_64k": 13, "xbot": 14}[case])
    for i in np.nonzero(v["up"])[0][:4096]:
        row = v["pas"][i][: v["pas_n"][i]]
        assert (np.diff(tab[row].astype(int)) >= 0).all(), i
