"""CPU tests of the oracle: RNG known-answer vectors and the reference's own
behavioural invariants for HyParView/Plumtree (no GPU needed)."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import _scenarios as S
from _oracle import Oracle, load
from partisan_amd import workloads as W
from partisan_amd.sim import default_config

NONE = 0xFFFFFFFF

HERE = os.path.dirname(os.path.abspath(__file__))


def test_philox_known_answers():
    """Philox4x32-10 against the published Random123 KAT vectors."""
    lib = load()
    kat = json.load(open(os.path.join(HERE, "golden", "philox4x32_10_kat.json")))
    out = (C.c_uint32 * 4)()
    for v in kat["vectors"]:
        lib.orc_philox(*v["ctr"], *v["key"], out)
        assert list(out) == v["out"]


def test_bucket_order_is_stable_hash():
    lib = load()
    b = [lib.orc_bucket16(i) for i in range(4096)]
    assert set(b) == set(range(16))
    counts = np.bincount(b, minlength=16)
    assert counts.min() > 4096 / 16 * 0.7


def test_config_a_connected_and_symmetric():
    """hyparview_membership_check/1 (test/partisan_SUITE.erl:2044-2108): the
    active-view digraph is strongly connected and symmetric."""
    sim, st = S.config_a(Oracle)
    v = sim.nodes()
    adj = S.active_graph(v)
    assert len(adj) == 32
    assert S.connected(adj)
    assert S.asymmetric(adj) == []
    assert (v["act_n"] <= 6).all() and (v["pas_n"] <= 30).all()
    assert st["overflow"].sum() == 0


def test_config_a_broadcast_reaches_everyone():
    """check_forward_message/3 with broadcast (partisan_SUITE.erl:1955-1994)."""
    sim, st = S.config_a(Oracle)
    v = sim.nodes()
    assert ((v["have"] >> 7) & 1).all()
    assert st["first_deliveries"].sum() == 31
    assert v["trk_hop"][0] == 0 and (v["trk_hop"][1:] >= 1).all()


def test_deterministic():
    _, a = S.doubling(Oracle, 512, 4, 40)
    _, b = S.doubling(Oracle, 512, 4, 40)
    S.compare_stats(a, b)
    _, c = S.doubling(Oracle, 512, 5, 40)
    assert not np.array_equal(a["digest"], c["digest"])


def test_stopped_members_leave_active_views():
    """hyparview_check_stopped_member/2 (partisan_SUITE.erl:2024-2041)."""
    sim, st, victims = S.crash_only(Oracle)
    v = sim.nodes()
    dead = set(victims.tolist())
    for i in range(len(v)):
        if v["up"][i]:
            assert not (set(v["act"][i][: v["act_n"][i]].tolist()) & dead), i
    adj = S.active_graph(v)
    assert S.connected(adj)
    assert st["exits"].sum() > 0


def test_revived_nodes_restart_without_join():
    """psim_revive: restarted without a join, a node comes back with init/1
    state (only itself active, empty passive view, start round = the restart)
    and is reached only by a node that still holds it in its passive view and
    promotes it (NEIGHBOR_REQUEST, hv:975-1053).  EXIT removed it from every
    holder's views and a full active view never promotes, so in this run all
    of them stay isolated -- the reference's behaviour for a restarted
    manager that is not told to join.  The rest of the overlay stays
    connected and symmetric, and the broadcast after the restart reaches
    every linked node and no isolated one."""
    sim, st, victims = S.crash_revive(Oracle)
    v = sim.nodes()
    assert v["up"][victims].all()
    assert (v["start_round"][victims] == 50).all()
    assert (v["act_n"][victims] == 1).all() and (v["act"][victims, 0] == victims).all()
    adj = S.active_graph(v)
    linked = {i: p for i, p in adj.items() if p}
    assert len(linked) == len(v) - len(victims)
    assert S.connected(linked)
    assert not S.asymmetric(linked)
    got = (v["have"] & 1).astype(bool)
    assert all(got[i] for i in linked), "broadcast missed a linked node"
    assert not got[victims].any()


def test_churn_partition_invariants():
    sim, st = S.churn_partition(Oracle, n=1024)
    v = sim.nodes()
    adj = S.active_graph(v)
    assert S.connected(adj)
    assert len(S.asymmetric(adj)) < len(adj) // 20
    # partition: no message crosses groups while it is in force
    assert st["overflow"].sum() == 0


def test_large_overlay_broadcast_reliability():
    sim, st = S.doubling(Oracle, 1 << 13, 11, 60)
    sim.broadcast(0, 3)
    st2 = sim.step(40)
    v = sim.nodes()
    assert ((v["have"] >> 3) & 1).mean() == 1.0
    hist = np.bincount(v["act_n"])
    assert hist[:3].sum() < 0.01 * len(v)    # almost every node keeps >= 2 peers
    assert st2["emitted"][:, 9].sum() >= len(v) - 1


def test_star_hotspot():
    """All nodes JOIN node 0 in one round: a 255-message inbox at one node.
    (The overlay may split into islands, as the reference would without the
    SUITE's sequential joins; only the absence of isolated nodes is asserted.)"""
    sim, st = S.star(Oracle, n=256)
    v = sim.nodes()
    assert (v["act_n"] >= 2).all()
    assert st["delivered"][:, 0].sum() == 255


def test_event_validation():
    sim = Oracle(default_config(n_nodes=16))
    with pytest.raises(Exception):
        sim.join(np.array([99], np.uint32), np.array([0], np.uint32))
    sim.broadcast(0, 1)
    with pytest.raises(Exception):
        sim.broadcast(0, 2)          # a second broadcast at the same root in one round
    with pytest.raises(Exception):
        sim.broadcast(1, 65)         # the message slot of id 1 (65 mod 64) is taken this round
    sim.broadcast(1, 2)              # another root: any node can broadcast


def test_duplicate_join_rejected():
    """A node starts at most once per round: a second psim_join of an id
    pending for the same round (in one batch or another call) is EINVAL and
    leaves the earlier joins in place (duplicates raced in k_join)."""
    sim = Oracle(default_config(n_nodes=16))
    with pytest.raises(Exception):
        sim.join(np.array([0, 3, 3], np.uint32), np.array([NONE, 0, 0], np.uint32))
    sim.join(np.array([0, 3], np.uint32), np.array([NONE, 0], np.uint32))
    with pytest.raises(Exception):
        sim.join(np.array([3], np.uint32), np.array([0], np.uint32))
    sim.step(1)
    sim.join(np.array([3], np.uint32), np.array([0], np.uint32))   # a later round: a restart
    sim.step(3)
    assert sim.nodes(3, 1)["up"][0] == 1


def test_multi_root_plumtree():
    """Four roots broadcasting together every 10 rounds for 200 rounds (68
    message ids, past the 64 message slots): every node keeps a per-root
    eager / lazy set for each root (pt:76-84, :599-631) with no overflow,
    each broadcast reaches (nearly) every node, and the per-root sets are
    ordsets sharing a pool of PSIM_PT_SET_POOL entries."""
    sim, st, roots = S.multi_root(Oracle, n=2048, roots=4, rounds=200)
    assert int(st["overflow"].sum()) == 0
    v = sim.nodes()
    used = v["pt_root"] != 0xFFFFFFFF
    assert used.sum(1).max() == 4
    got = {int(r) for r in np.unique(v["pt_root"][used])}
    assert got <= {r | 0x80000000 for r in roots}
    for i in range(0, 2048, 97):
        o = 0
        for k in range(4):                 # pooled: slot k follows slots 0..k-1
            ne = int(v["pt_eager_n"][i][k])
            e = [int(x) for x in v["pt_eager"][i][o:o + ne]]
            assert e == sorted(set(e))
            o += ne
        assert o <= 64 and not v["pt_eager"][i][o:].any()
    # 68 broadcasts, each delivered to nearly all 2048 nodes
    assert int(st["first_deliveries"].sum()) > 0.98 * 68 * 2047


def test_plumtree_off():
    sim, st = S.doubling(Oracle, 256, 2, 30, plumtree=0)
    assert st["emitted"][:, 9:14].sum() == 0
    assert S.connected(S.active_graph(sim.nodes()))


def test_partition_groups_0_to_254():
    """psim_set_partition takes groups 0..PSIM_PARTITION_MAX (254): 255 is
    the engine's down mark in its one-byte up-and-partition pairs"""
    from partisan_amd.sim import SimError
    n = 64
    sim = Oracle(default_config(n_nodes=n, seed=3))
    g = np.full(n, 254, np.uint8)
    sim.set_partition(g)
    g[5] = 255
    with pytest.raises(SimError):
        sim.set_partition(g)


def test_partition_blocks_cross_traffic():
    n = 512
    sim = Oracle(default_config(n_nodes=n, seed=3))
    sim.run_schedule(W.doubling_join(n, 3), 40)
    g = W.half_partition(n)
    sim.set_partition(g)
    sim.step(1)
    sim.broadcast(0, 2)
    sim.step(30)
    v = sim.nodes()
    got = (v["have"] >> 2) & 1
    assert got[: n // 2].mean() > 0.2      # the root side reaches part of its group
    assert got[n // 2:].sum() == 0


def _golden():
    return json.load(open(os.path.join(HERE, "golden", "oracle_traces.json")))["traces"]


@pytest.mark.parametrize("name", sorted(json.load(open(os.path.join(HERE, "golden", "oracle_traces.json")))["traces"]))
def test_oracle_matches_committed_traces(name):
    """tests/golden/oracle_traces.json (self-generated by
    tests/golden/gen_oracle_traces.py): per-round digests and the final state
    hash of each scenario; pins the oracle against unintended change."""
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import gen_oracle_traces as G
    got, want = G.trace(name), _golden()[name]
    assert got["digest"] == want["digest"]
    assert got["emitted"] == want["emitted"]
    assert got["state_sha256"] == want["state_sha256"]
    # the rounds an earlier oracle change left untouched still hold
    guards = json.load(open(os.path.join(HERE, "golden", "oracle_traces.json"))).get("guards", {})
    for g in guards.get(name, []):
        assert got["digest"][:g["rounds"]] == g["digest"], g["changed_by"]


def _py_histograms(sim):
    """The overlay statistics restated from the node views (Python)."""
    v = sim.nodes()
    have, rnd, hop = sim.delivery()
    n = len(v)
    up = v["up"].astype(bool)
    B = 64
    hist = {k: np.zeros(B, np.uint64) for k in ("active_in", "passive_in", "active_out", "passive_fill", "hop")}
    ina = np.zeros(n, np.int64)
    inp = np.zeros(n, np.int64)
    links = sym = 0
    parent = list(range(n))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x
    acts = {i: [int(p) for p in v["act"][i][: v["act_n"][i]] if p != i] for i in range(n)}
    for i in range(n):
        if not up[i]:
            continue
        hist["active_out"][min(len(acts[i]), B - 1)] += 1
        hist["passive_fill"][min(int(v["pas_n"][i]), B - 1)] += 1
        for p in acts[i]:
            if up[p]:
                ina[p] += 1
                links += 1
                sym += i in acts[p]
                a, b = find(i), find(p)
                if a != b:
                    parent[max(a, b)] = min(a, b)
        for p in v["pas"][i][: v["pas_n"][i]]:
            if p != i and up[p]:
                inp[p] += 1
        if have[i]:
            hist["hop"][min(int(hop[i]), B - 1)] += 1
    comps = {}
    for i in range(n):
        if up[i]:
            hist["active_in"][min(ina[i], B - 1)] += 1
            hist["passive_in"][min(inp[i], B - 1)] += 1
            comps[find(i)] = comps.get(find(i), 0) + 1
    return hist, links, sym, len(comps), max(comps.values()), int((have.astype(bool) & up).sum())


def test_histograms_match_views():
    """psim_get_histograms (oracle) against the same statistics restated in
    Python from psim_get_nodes / psim_get_delivery, after a doubling
    bootstrap with a broadcast and a few crashes (SURVEY 8(d) config C/D
    report: in-degree histograms, passive fill, connectivity, reliability,
    last-delivery hop)."""
    n = 1024
    sim, _ = S.doubling(Oracle, n, 7, 60, bcast_period=20, bcast_first=30)
    sim.crash(np.arange(0, n, 97, dtype=np.uint32))
    sim.step(3)
    h = sim.histograms()
    hist, links, sym, comps, largest, deliv = _py_histograms(sim)
    for k, a in hist.items():
        assert (h[k] == a).all(), k
    assert h["n_up"] == int(sim.nodes()["up"].sum())
    assert (h["active_links"], h["symmetric_links"], h["components"], h["largest_component"]) == \
        (links, sym, comps, largest)
    assert h["delivered"] == deliv
    assert h["components"] == 1 and h["delivered"] > 0.9 * h["n_up"]


def test_message_conservation():
    """Every record emitted in round r is delivered or dropped in round r + 1
    (under churn and multi-root broadcasts): the identity bench.py reports as
    `conservation` for the GPU window."""
    _, st, _ = S.multi_root(Oracle, n=1024, rounds=120, churn=True)
    em = st["emitted"].sum(axis=1)
    got = st["delivered"].sum(axis=1) + st["dropped"]
    assert em.sum() > 0 and np.array_equal(em[:-1], got[1:])


def _conn_invariants(v):
    """The connection table of every live node (App. A Q11): lingering peers
    are running peers outside the active view; entries marked PSIM_CONN_DOWN
    are active members (without a connection); no duplicates."""
    from partisan_amd import _abi
    up = v["up"].astype(bool)
    n_ling = 0
    for i in np.nonzero(up)[0]:
        k = int(v["conn_n"][i])
        assert k <= _abi.CONN_CAP
        ent = [int(x) for x in v["conn"][i][:k]]
        assert len(set(ent)) == k
        assert all(x == 0 for x in v["conn"][i][k:])
        act = set(int(x) for x in v["act"][i][: v["act_n"][i]])
        for e in ent:
            p = e & ~_abi.CONN_DOWN
            if e & _abi.CONN_DOWN:
                assert p in act, (i, e)
            else:
                assert p not in act and p != i and up[p], (i, e)
                n_ling += 1
    return n_ling


def test_connection_table_invariants():
    """Lingering connections: after churn + a partition
    every table entry obeys the model, some nodes hold lingering peers, and
    none overflowed (PSIM_CONN_CAP)."""
    sim, st = S.churn_partition(Oracle, n=2048)
    assert _conn_invariants(sim.nodes()) > 0
    assert int(st["overflow_by"][:, 4].sum()) == 0


def test_lingering_exits_prune_every_holder():
    """A crash reaches every holder of a connection -- lingering ones too --
    so the crashed peer leaves every passive view and every table in that
    round (hyparview:609-654)."""
    n = 2048
    sim, _ = S.churn_partition(Oracle, n=n)
    v = sim.nodes()
    holders = {}
    for i in np.nonzero(v["up"])[0]:
        for e in v["conn"][i][: v["conn_n"][i]]:
            if not int(e) & 0x80000000:
                holders.setdefault(int(e), []).append(int(i))
    victims = sorted(holders, key=lambda p: -len(holders[p]))[:16]
    assert victims
    sim.crash(np.array(victims, np.uint32))
    st = sim.step(1)
    w = sim.nodes()
    vs = set(victims)
    for i in np.nonzero(w["up"])[0]:
        assert not vs & set(int(x) for x in w["conn"][i][: w["conn_n"][i]])
    # (a passive view may take a victim back in the same round from an
    # exchange already in flight, so only the EXITs are counted here)
    assert int(st["exits"].sum()) >= sum(len(holders[p]) for p in victims)


def test_msg_slots_and_strict_capacity():
    """psim_get_msg_slots names the id and root owning each message slot; with
    cfg.strict a fixed-table overflow -- here a fifth live Plumtree root at a
    node (PSIM_PT_ROOTS = 4, the heartbeat case of plumtree_backend:179-200)
    -- fails the step loudly instead of being counted."""
    from partisan_amd import _abi
    from partisan_amd.sim import SimError
    sim, st, roots = S.multi_root(Oracle, n=512, roots=6, rounds=60)
    ids, rts = sim.msg_slots()
    live = ids != _abi.PSIM_NONE
    assert live.sum() > 0 and all(int(i) % _abi.MSG_SLOTS == k for k, i in enumerate(ids) if i != _abi.PSIM_NONE)
    assert set(int(r) & ~_abi.PSIM_MAP_BIT for r in rts[live]) <= set(roots)
    assert int(st["overflow_by"][:, 2].sum()) > 0             # counted (strict = 0)
    with pytest.raises(SimError, match="ECAPACITY"):
        S.multi_root(Oracle, n=512, roots=6, rounds=60, strict=1)
    _, st4, _ = S.multi_root(Oracle, n=512, roots=4, rounds=60, strict=1)   # four roots fit
    assert int(st4["overflow"].sum()) == 0


def test_heartbeat_fails_loudly_when_strict():
    """More live Plumtree roots than a node's slots: counted by default,
    PSIM_ECAPACITY with cfg.strict (no silent protocol change)."""
    from partisan_amd.sim import SimError
    _, st = S.heartbeat(Oracle)
    assert int(st["overflow"].sum()) > 0
    with pytest.raises(SimError, match="ECAPACITY"):
        S.heartbeat(Oracle, strict=1)


def _views_in_bucket_order(v, tab):
    for i in np.nonzero(v["up"])[0]:
        for f, nf in (("act", "act_n"), ("pas", "pas_n")):
            row = v[f][i][: v[nf][i]]
            b = tab[row]
            assert (np.diff(b.astype(int)) >= 0).all(), (i, f, row.tolist(), b.tolist())


def test_bucket_table_sets_view_order():
    """App. A Q1: with a table installed (psim_set_bucket_table) every view
    is in sets:to_list order of that table -- ascending bucket -- and the run
    differs from the stand-in's; the stand-in's own table reproduces the
    default run bit for bit."""
    tab = S.random_buckets(32, 7)
    sim, st = S.config_a(S.with_buckets(Oracle, table=tab))
    _views_in_bucket_order(sim.nodes(), tab)
    assert S.connected(S.active_graph(sim.nodes()))
    base, bst = S.config_a(Oracle)
    assert not np.array_equal(st["digest"], bst["digest"])
    lib = load()
    own = np.array([lib.orc_bucket16(i) for i in range(32)], np.uint8)
    same, sst = S.config_a(S.with_buckets(Oracle, table=own))
    S.compare_stats(sst, bst)
    S.compare_nodes(same.nodes(), base.nodes())
    _views_in_bucket_order(base.nodes(), own)


def test_bucket_table_scamp_v1_order():
    """SCAMP v1's membership is a sets v1 set too (scamp_v1:45-279): its
    view follows the table (views of <= 80 entries)."""
    n = 512
    tab = S.random_buckets(n, 3)
    sim, _ = S.pl_doubling(S.with_buckets(Oracle, table=tab), n, 5, 40, 1)
    v = sim.strategy_nodes()
    for i in range(n):
        row = v["view"][i][: v["view_n"][i]]
        if 0 < len(row) <= 80:
            assert (np.diff(tab[row].astype(int)) >= 0).all(), i


def test_bucket_table_checks():
    from partisan_amd.sim import SimError
    sim = Oracle(default_config(n_nodes=32))
    with pytest.raises(SimError):
        sim.set_bucket_table(np.full(32, 16, np.uint8))      # buckets are 0..15
    with pytest.raises(SimError):
        sim.set_bucket_table(np.zeros(31, np.uint8))          # one per node
    sim.set_bucket_table(np.zeros(32, np.uint8))
    sim.set_bucket_table(None)
    sim.step(1)
    with pytest.raises(SimError):
        sim.set_bucket_table(np.zeros(32, np.uint8))          # before the first round only
