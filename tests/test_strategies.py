"""CPU tests of the pluggable-manager strategies in the oracle (SURVEY 8(a)
s1-s4): the reference's own assertions for them, restated over the round
model R0-P.

- membership agreement (test/prop_partisan.erl:944-967): with the full
  strategy every live node ends with the same member set, all started nodes;
- connectivity_test / check_forward_message (test/partisan_SUITE.erl
  :1214-1259, :1955-1994): every node's members are reachable -- the overlay
  the SCAMP views span is connected and holds only started nodes;
- scamp v2 keep_subscription (scamp_v2:284-338): X in in_view(Y) => Y in
  partial_view(X).
Parity against the Erlang modules is unpinned (no VM here)."""
import numpy as np
import pytest

import _scenarios as S
from _oracle import Oracle
from partisan_amd.sim import default_config

NONE = 0xFFFFFFFF


def _views(sim):
    v = sim.strategy_nodes()
    return {i: [int(x) for x in v["view"][i][: v["view_n"][i]]] for i in range(len(v)) if v["up"][i]}


def _weakly_connected(adj):
    if not adj:
        return True
    und = {i: set() for i in adj}
    for i, vs in adj.items():
        for j in vs:
            if j in und and j != i:
                und[i].add(j)
                und[j].add(i)
    start = next(iter(und))
    seen, stack = {start}, [start]
    while stack:
        x = stack.pop()
        for y in und[x] - seen:
            seen.add(y)
            stack.append(y)
    return len(seen) == len(und)


@pytest.mark.parametrize("fanout", [0, 5])
def test_full_membership_agreement(fanout):
    n = 16 if fanout == 0 else 2048
    sim, st = S.pl_doubling(Oracle, n, 3, 60, strategy=0, fanout=fanout)
    v = sim.strategy_nodes()
    assert (v["members"] == n).all()
    assert len(set(v["members_hash"].tolist())) == 1
    assert sim.members(5) == list(range(n))
    assert st["overflow"].sum() == 0
    # the handshake: one HELLO and one STATE per joiner
    assert st["emitted"][:, 0].sum() == n - 1 and st["delivered"][:, 1].sum() == n - 1


def test_full_fanout_bounds_messages():
    n = 4096
    sim, st = S.pl_doubling(Oracle, n, 5, 60, strategy=0, fanout=5)
    # coalesced gossip: at most one gossip of `fanout` messages per node and round
    assert (st["emitted"][:, 2] <= 5 * n).all()
    assert (sim.strategy_nodes()["members"] == n).all()


def test_full_crashed_members_stay_members():
    """no leave: a crashed node stays in every ORSet, sends to it fail"""
    n = 1024
    sim, st = S.pl_doubling(Oracle, n, 4, 80, strategy=0, fanout=5, crash_at=40)
    v = sim.strategy_nodes()
    assert (v["members"] == n).all()
    assert st["send_fail"][41:].sum() > 0


def test_full_restart_rejected():
    sim = Oracle(default_config(n_nodes=8, manager=1, strategy=0))
    sim.join(np.array([0], np.uint32), np.array([NONE], np.uint32))
    with pytest.raises(Exception):
        sim.join(np.array([0], np.uint32), np.array([NONE], np.uint32))


@pytest.mark.parametrize("strategy", [1, 2])
def test_scamp_views_connected(strategy):
    n = 2048
    sim, st = S.pl_doubling(Oracle, n, 6, 120, strategy=strategy)
    views = _views(sim)
    assert len(views) == n
    assert _weakly_connected(views)
    assert all(0 <= j < n for vs in views.values() for j in vs)
    assert all(i in vs for i, vs in views.items())      # myself() stays a member
    assert st["overflow"].sum() == 0
    assert (sim.strategy_nodes()["pending"] == NONE).all()


def test_scamp_v2_in_view_consistent():
    n = 1024
    sim, st = S.pl_doubling(Oracle, n, 8, 100, strategy=2)
    v = sim.strategy_nodes()
    for y in range(n):
        for x in v["in_view"][y][: v["in_n"][y]]:
            assert y in v["view"][x][: v["view_n"][x]], (x, y)


def test_scamp_v1_set_order_and_no_duplicates():
    n = 1024
    sim, _ = S.pl_doubling(Oracle, n, 2, 80, strategy=1)
    from _oracle import load
    lib = load()
    for i, vs in _views(sim).items():
        assert len(set(vs)) == len(vs)
        b = [lib.orc_bucket16(x) for x in vs]
        assert b == sorted(b), i                        # sets:to_list/1 bucket order


@pytest.mark.parametrize("strategy", [1, 2])
def test_scamp_churn_partition(strategy):
    n = 1024
    sim, st = S.pl_doubling(Oracle, n, 9, 120, strategy=strategy, crash_at=50, part_at=70)
    assert st["send_fail"].sum() > 0
    v = sim.strategy_nodes()
    assert v["up"].all()
    assert _weakly_connected(_views(sim))


@pytest.mark.parametrize("strategy", [0, 1, 2])
def test_leave_stops_like_a_crash(strategy):
    """leave/0 under the pluggable manager (pluggable:502-515, :1390-1420):
    the Strategy:leave/2 messages are casts to the manager itself, lost when
    it stops, so the run is identical to crashing the same nodes."""
    n = 1024
    kw = dict(strategy=strategy, fanout=5 if strategy == 0 else 0, crash_at=40, part_at=60)
    _, a = S.pl_doubling(Oracle, n, 11, 90, leave=True, **kw)
    _, b = S.pl_doubling(Oracle, n, 11, 90, **kw)
    S.compare_stats(a, b)
    assert a["send_fail"][41:].sum() > 0


def test_scamp_v2_remote_leave_stops_exactly_the_targets():
    """leave/1 under SCAMP v2: {bootstrap_remove_subscription, T} reaches T
    (it is in the actor's partial view), which stops (scamp_v2:192-238);
    nobody else changes state because of it."""
    n = 1024
    sim, st, actors, targets = S.pl_leave_remote(Oracle, n, 5, 60, strategy=2)
    up = sim.strategy_nodes()["up"].astype(bool)
    down = set(np.nonzero(~up)[0].tolist())
    assert down == set(targets.tolist())
    assert st["emitted"][40, 7] > 0 and st["delivered"][41, 7] == st["emitted"][40, 7]


def test_scamp_v1_remote_leave_crashes_every_holder():
    """leave/1 under SCAMP v1: {remove_subscription, T} to the actor's old
    membership; every receiver holding T crashes on the swapped
    sets:del_element/2 arguments (App. A Q12), T itself included, and the
    actor's view no longer holds T."""
    n = 1024
    sim, st, actors, targets = S.pl_leave_remote(Oracle, n, 6, 60, strategy=1)
    v = sim.strategy_nodes()
    up = v["up"].astype(bool)
    assert not up[targets].any()
    assert (~up).sum() >= len(targets)
    for x, t in zip(actors, targets):
        if up[x]:
            assert t not in v["view"][x][: v["view_n"][x]]
    # a stopped manager's round sends nothing: emitted == delivered + dropped next round
    em = st["emitted"].sum(1)
    assert (em[40:-1] == st["delivered"].sum(1)[41:] + st["dropped"][41:]).all()


@pytest.mark.parametrize("fanout", [0, 5])
def test_full_remote_leave_tombstones(fanout):
    """leave/1 under the full strategy (full:58-89): the actor tombstones the
    target's add and gossips; the removal spreads by merge (adds and removes
    OR-ed) until every running member agrees on n - k members; with the
    reference's gossip-to-all (fanout 0) every target gets the actor's
    gossip, finds itself removed and stops (pluggable:1182-1188)."""
    n = 32 if fanout == 0 else 1024          # fanout 0: |members| messages per gossip
    sim, st, actors, targets = S.pl_leave_remote(Oracle, n, 3, 90, strategy=0, fanout=fanout, k=4)
    v = sim.strategy_nodes()
    up = v["up"].astype(bool)
    if fanout == 0:
        assert not up[targets].any()
        assert up.sum() == n - len(targets)
    others = up.copy()
    others[targets] = False                 # (fanout 5: a target nobody gossiped to yet runs on)
    assert (v["members"][others] == n - len(targets)).all()
    bits = sim.member_bits(int(np.nonzero(others)[0][0]))
    ids = {i for i in range(n) if (int(bits[i >> 5]) >> (i & 31)) & 1}
    assert not ids & set(targets.tolist())


def test_leave_node_rejections():
    hv = Oracle(default_config(n_nodes=8))
    with pytest.raises(Exception):
        hv.leave_node(np.array([1], np.uint32), np.array([2], np.uint32))
    sv = Oracle(default_config(n_nodes=8, manager=1, strategy=1))
    with pytest.raises(Exception):     # one leave/1 call per actor and round
        sv.leave_node(np.array([1, 1], np.uint32), np.array([2, 3], np.uint32))
    with pytest.raises(Exception):
        sv.leave_node(np.array([1], np.uint32), np.array([9], np.uint32))


def test_hyparview_leave_is_an_error():
    """hyparview:363-364: handle_call({leave, _}) replies `error`"""
    sim = Oracle(default_config(n_nodes=8))
    with pytest.raises(Exception):
        sim.leave(np.array([1], np.uint32))


def test_pluggable_rejects_broadcast():
    sim = Oracle(default_config(n_nodes=8, manager=1, strategy=1))
    with pytest.raises(Exception):
        sim.broadcast(0, 1)


# ---------------------------------------------------------------- omission faults
# The crash-fault model's omissions (prop_partisan_crash_fault_model:93-229)
# through the pluggable manager's interposition funs (pluggable:297-326,
# :634-836): a dropped send never reaches the connection lookup or the
# dispatch draw, a dropped receive is never handled.

@pytest.mark.parametrize("strategy,fanout", [(0, 5), (1, 0), (2, 0)])
def test_omission_faults_drop_and_heal(strategy, fanout):
    n = 1024
    sim, st, f = S.pl_omission(Oracle, n, 21, 120, strategy, fanout)
    assert st["omitted"][:40].sum() == 0
    assert st["omitted"][40:75].sum() > 0
    assert st["omitted"][76:].sum() == 0                  # healed (resolve_all_faults_with_heal)
    assert st["overflow"].sum() == 0
    if strategy == 0:                                     # the ORSet converges again after the heal
        v = sim.strategy_nodes()
        assert (v["members"] == n).all()
    else:
        assert _weakly_connected(_views(sim))


def test_omission_that_never_matches_changes_nothing():
    """installed funs whose pairs never carry a message (and a general
    omission of nodes that never start) leave the run bit-identical"""
    n = 1024

    def quiet(make):
        sim = make(default_config(n_nodes=n + 8, seed=4, manager=1, strategy=2))
        ghosts = np.arange(n, n + 8, dtype=np.uint32)      # never started

        def hook(r):
            if r == 30:
                sim.begin_omission(ghosts)
                sim.begin_send_omission(ghosts, ghosts[::-1].copy())
                sim.begin_receive_omission(np.zeros(8, np.uint32), ghosts)
        return sim.run_schedule(S.W.doubling_join(n, 4), 80, extra=hook)

    def plain(make):
        sim = make(default_config(n_nodes=n + 8, seed=4, manager=1, strategy=2))
        return sim.run_schedule(S.W.doubling_join(n, 4), 80)
    S.compare_stats(quiet(Oracle), plain(Oracle))


def test_general_omission_silences_a_node():
    """begin_omission at x: x sends no strategy message and handles none
    (full strategy, reference gossip-to-all on 16 nodes): its member set
    stops growing and nobody learns of it (its join gossip never leaves),
    while the others agree on the rest; after end_omission all converge."""
    n = 16
    sim = Oracle(default_config(n_nodes=n, seed=2, manager=1, strategy=0))
    x = np.array([9], np.uint32)
    sched = S.W.doubling_join(n, 2)
    # node 9 starts in round 4 (ids [8, 16)); silence it from round 5
    st = sim.run_schedule(sched, 5)
    sim.begin_omission(x)
    st = sim.step(40)
    v = sim.strategy_nodes()
    assert st["omitted"].sum() > 0
    assert v["members"][9] < n
    assert (np.delete(v["members"], 9) == n - 1).all()
    sim.end_omission(x)
    sim.step(30)
    assert (sim.strategy_nodes()["members"] == n).all()


def test_send_omission_counts_and_draws():
    """a send omission costs no dispatch draw: the sender's draw counter
    runs behind the same run without the fault by exactly the omitted count
    when nothing else differs (SCAMP v1 pings to one omitted member)"""
    n = 64
    base = Oracle(default_config(n_nodes=n, seed=6, manager=1, strategy=1))
    flt = Oracle(default_config(n_nodes=n, seed=6, manager=1, strategy=1))
    for sim in (base, flt):
        sim.run_schedule(S.W.doubling_join(n, 6), 30)
    v = base.strategy_nodes()
    x = next(i for i in range(n) if v["view_n"][i] >= 3)
    y = int([j for j in v["view"][x][: v["view_n"][x]] if j != x][0])
    flt.begin_send_omission(np.array([x], np.uint32), np.array([y], np.uint32))
    # one periodic round of x (periodic every 10 rounds from its start)
    a, b = base.step(1), flt.step(1)
    while a["omitted"].sum() == b["omitted"].sum() == 0 and base.round < 60:
        a, b = base.step(1), flt.step(1)
    assert b["omitted"].sum() >= 1
    ra, rb = base.strategy_nodes()["rng_ctr"][x], flt.strategy_nodes()["rng_ctr"][x]
    assert ra - rb == b["omitted"].sum()


def test_omission_rejections():
    hv = Oracle(default_config(n_nodes=8))
    with pytest.raises(Exception):                        # HyParView: no interposition layer
        hv.begin_omission(np.array([1], np.uint32))
    sv = Oracle(default_config(n_nodes=8, manager=1, strategy=1))
    with pytest.raises(Exception):
        sv.begin_send_omission(np.array([1], np.uint32), np.array([8], np.uint32))
