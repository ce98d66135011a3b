"""Event scripts shared by the oracle tests and the GPU parity tests.  Each
scenario drives any `_Driver` (GPU Simulator or CPU Oracle) through the same
API calls, so two backends can be compared round by round."""
import numpy as np

from partisan_amd import workloads as W
from partisan_amd.sim import default_config

STAT_FIELDS = ["emitted", "delivered", "dropped", "nodes_up", "nodes_processed", "exits",
               "send_fail", "first_deliveries", "overflow", "overflow_by", "digest", "omitted"]


def random_buckets(n, seed):
    """A sets v1 bucket table (0..15 per node) unrelated to the built-in
    stand-in: what an in-BEAM harness export of erlang:phash(NodeSpec, 16)
    looks like to the engine (psim_set_bucket_table)."""
    return np.random.Generator(np.random.PCG64([seed, 0xB16])).integers(0, 16, n).astype(np.uint8)


def with_buckets(make, seed=7, table=None):
    """`make` with a bucket table installed before the first round."""
    def mk(cfg):
        sim = make(cfg)
        sim.set_bucket_table(random_buckets(cfg.n_nodes, seed) if table is None else table)
        return sim
    return mk


def _bcast_every(sim, period, first, root=0, count=None):
    state = {"k": 0}

    def hook(r):
        if r >= first and (r - first) % period == 0 and (count is None or state["k"] < count):
            sim.broadcast(root, state["k"] % 0x10000)
            state["k"] += 1
    return hook


def config_a(make, seed=1, rounds=200, tail=40):
    """Config A: 32 nodes join node 0 one per round, 200 rounds, then one
    broadcast from node 0 (test/partisan_SUITE.erl:1591-1601, :2044-2108)."""
    sim = make(default_config(n_nodes=32, seed=seed))
    st = [sim.run_schedule(W.sequential_join(32), rounds)]
    sim.broadcast(0, 7)
    st.append(sim.step(tail))
    return sim, np.concatenate(st)


def doubling(make, n, seed, rounds, bcast_period=None, bcast_first=None, **cfg):
    sim = make(default_config(n_nodes=n, seed=seed, **cfg))
    hook = None
    if bcast_period:
        hook = _bcast_every(sim, bcast_period, bcast_first)
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st


def multistep(make, n=4096, seed=9):
    """Rounds run several at a time between events (psim_step(k), k > 1),
    so the rank path runs batches of rounds (run_batch_ranked) whose
    fixed-size exchange was sized by quieter rounds: a broadcast after a
    quiet stretch, a crash wave, a partition -- each a step in the message
    counts that overflows a capacity and makes every rank redo that round
    exactly.  Doubling bootstrap, then 40 quiet rounds, a broadcast and 30
    rounds, 5 % crashes and 20 rounds, a half/half partition for 12 rounds,
    a broadcast and 25 rounds."""
    sim = make(default_config(n_nodes=n, seed=seed))
    st = [sim.run_schedule(W.doubling_join(n, seed), 20)]
    st.append(sim.step(40))
    sim.broadcast(0, 1)
    st.append(sim.step(30))
    rng = np.random.Generator(np.random.PCG64([seed, 77]))
    victims = np.sort(rng.choice(np.arange(1, n, dtype=np.uint32), size=n // 20, replace=False)).astype(np.uint32)
    sim.crash(victims)
    st.append(sim.step(20))
    sim.set_partition(W.half_partition(n))
    st.append(sim.step(12))
    sim.clear_partition()
    sim.broadcast(1, 2)
    st.append(sim.step(25))
    return sim, np.concatenate(st)


def churn_partition(make, n=2048, seed=5, rounds=140, **cfg):
    """Config E in miniature: doubling bootstrap, 20% churn over rounds
    40-79, a half/half partition for rounds 90-99, a broadcast every 10."""
    sim = make(default_config(n_nodes=n, seed=seed, **cfg))
    churn = {r: (v, c) for r, v, c in W.churn_schedule(n, seed, 0.2, 40, 40)}
    part = W.half_partition(n)
    bc = _bcast_every(sim, 10, 30)

    def hook(r):
        if r in churn:
            v, c = churn[r]
            sim.crash(v)
            sim.join(v, c)
        if r == 90:
            sim.set_partition(part)
        if r == 100:
            sim.clear_partition()
        bc(r)
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st


def xbot_churn(make, n=2048, seed=5, rounds=140, period=10):
    """churn_partition under the X-BOT manager: optimization
    rounds every `period` rounds through the churn and the partition."""
    return churn_partition(make, n=n, seed=seed, rounds=rounds, manager=2, xbot_period=period)


def joiner_crash(make, n=2048, seed=3, rounds=40, **cfg):
    """A doubling bootstrap where a third of each round's joiners crash two
    rounds after they start, while their FORWARD_JOINs are still walking.
    With arwl = prwl (the variant config) the first hop inserts the joiner
    into the passive view (hv:859-863) and, when no forward target exists and
    the joiner is unreachable, the reference discards that insert
    (hv:896-897, {error, not_found} -> State0): ~600 such reverts per run."""
    sim = make(default_config(n_nodes=n, seed=seed, **cfg))

    def hook(r):
        if r >= 3 and (1 << (r - 3)) < n:
            ids = np.arange(1 << (r - 3), min(n, 1 << (r - 2)), dtype=np.uint32)
            sim.crash(ids[::3])
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st


def heartbeat(make, n=64, seed=23, rounds=120, period=10, first=40, **cfg):
    """plumtree_backend's heartbeat (backend:179-200, :221-228): every live
    node broadcasts {mynode(), unique_integer} every `period` rounds, so every
    node is a root (p8).  Each node beats at its own phase (id mod period);
    message ids count up and wrap the 64 slots.  With more live roots than a
    node's PSIM_PT_ROOTS slots and more live ids than PSIM_MSG_SLOTS, the
    overflows are counted (cfg.strict = 0) or fail the step (strict = 1)."""
    sim = make(default_config(n_nodes=n, seed=seed, **cfg))
    state = {"k": 0}

    def hook(r):
        if r >= first:
            for root in range(n):
                if (r + root) % period == 0:
                    sim.broadcast(root, state["k"] % 0x10000)
                    state["k"] += 1
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st


def lingering_exits(make, n=2048, seed=5, extra_rounds=6, k=16):
    """churn_partition, then a crash of the k peers held by the most
    lingering connections: their EXITs reach holders
    outside their active views; then a few rounds more."""
    sim, st = churn_partition(make, n=n, seed=seed)
    v = sim.nodes()
    holders = {}
    for i in np.nonzero(v["up"])[0]:
        for e in v["conn"][i][: v["conn_n"][i]]:
            if not int(e) & 0x80000000:
                holders[int(e)] = holders.get(int(e), 0) + 1
    victims = sorted(holders, key=lambda p: (-holders[p], p))[:k]
    sim.crash(np.array(victims, np.uint32))
    sim.broadcast(1, 999)
    st2 = sim.step(extra_rounds)
    return sim, np.concatenate([st, st2]), victims


def e_miniature(make, n=1 << 14, seed=101, rounds=90):
    """Config E in miniature, as bench.py's built-in sharding check runs it:
    doubling bootstrap, 20% churn over rounds 30-49 (crash, restart and
    rejoin), a half/half partition for rounds 55-64, a broadcast from node 0
    every 10 rounds from round 20."""
    sim = make(default_config(n_nodes=n, seed=seed))
    ch = {r: (v, c) for r, v, c in W.churn_schedule(n, seed, 0.2, 30, 20)}

    def hook(r):
        if r in ch:
            sim.crash(ch[r][0])
            sim.join(ch[r][0], ch[r][1])
        if r == 55:
            sim.set_partition(W.half_partition(n))
        if r == 65:
            sim.clear_partition()
        if r >= 20 and r % 10 == 0:
            sim.broadcast(0, (r // 10) % 0x10000)
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st


def out_tail(make, n=512, seed=3, period=2, part_on=40, part_off=80, rounds=110, snap_at=(60, 79, 81)):
    """Plumtree outstanding tables past one 64-entry register (pt:574-579
    adds, :562-567 acks): a broadcast from node 0 every `period` rounds
    from round 30, and a half/half partition over rounds part_on..part_off
    - 1 that leaves the lazy pushes across it unacked (up to 88 entries on a
    node at the defaults, none dropped; period=1 fills tables to
    PSIM_PT_OUT_CAP and drops).  The heal acks them.  Returns the node
    views at the rounds in `snap_at` too (the tables at their largest)."""
    sim = make(default_config(n_nodes=n, seed=seed))
    snaps = {}
    state = {"k": 0}

    def hook(r):
        if r in snap_at:
            snaps[r] = sim.nodes()
        if r == part_on:
            sim.set_partition(W.half_partition(n))
        if r == part_off:
            sim.clear_partition()
        if r >= 30 and r % period == 0:
            sim.broadcast(0, state["k"] % 0x10000)
            state["k"] += 1
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st, snaps


VARIANT = dict(max_active_size=8, max_passive_size=20, arwl=6, prwl=6, persist_epoch=1)


def multi_root(make, n=2048, seed=17, rounds=160, roots=4, period=10, first=30, churn=False, **cfg):
    """Plumtree with several roots (pt:76-84 per-root eager/lazy sets,
    backend:179-200 heartbeat broadcasts): `roots` distinct nodes, drawn
    once, each originate a broadcast every `period` rounds from `first`, in
    the same round; message ids count up, past PSIM_MSG_SLOTS on long runs
    (old ids retire).  churn=True adds 10% crash + rejoin churn over rounds
    60-79.  With roots <= PSIM_PT_ROOTS every node keeps every root's sets
    (overflow 0); more roots exercise the full-slots path."""
    sim = make(default_config(n_nodes=n, seed=seed, **cfg))
    rng = np.random.Generator(np.random.PCG64([seed, 31]))
    rs = [int(x) for x in rng.choice(n, size=roots, replace=False)]
    ch = {r: (v, c) for r, v, c in W.churn_schedule(n, seed, 0.1, 60, 20, protect=tuple(rs))} if churn else {}
    state = {"k": 0}

    def hook(r):
        if r in ch:
            sim.crash(ch[r][0])
            sim.join(ch[r][0], ch[r][1])
        if r >= first and (r - first) % period == 0:
            for root in rs:
                sim.broadcast(root, state["k"] % 0x10000)
                state["k"] += 1
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st, rs


def crash_only(make, n=1024, seed=9, rounds=80):
    """Crashes without restarts: EXIT handling and the stopped-member check
    (test/partisan_SUITE.erl:2024-2041)."""
    sim = make(default_config(n_nodes=n, seed=seed))
    victims = np.arange(3, n, 17, dtype=np.uint32)

    def hook(r):
        if r == 40:
            sim.crash(victims)
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st, victims


def crash_revive(make, n=1024, seed=11, rounds=100):
    """Crashes at round 40, the same nodes restarted without a join at round
    50 (psim_revive: init/1 state, reached through other nodes' passive
    views), a broadcast at round 70."""
    sim = make(default_config(n_nodes=n, seed=seed))
    victims = np.arange(5, n, 13, dtype=np.uint32)
    bc = _bcast_every(sim, 1000, 70)

    def hook(r):
        if r == 40:
            sim.crash(victims)
        if r == 50:
            sim.revive(victims)
        bc(r)
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st, victims


def star(make, n=512, seed=3, rounds=60):
    sim = make(default_config(n_nodes=n, seed=seed))
    st = sim.run_schedule(W.star_join(n), rounds)
    sim.broadcast(0, 1)
    st2 = sim.step(30)
    return sim, np.concatenate([st, st2])


def pl_doubling(make, n, seed, rounds, strategy, fanout=0, crash_at=None, part_at=None, leave=False,
                **cfg):
    """The pluggable manager with one membership strategy (SURVEY 8(a)
    s1-s4): doubling bootstrap, then optional crashes (scamp: 10% of the
    nodes, restarted and rejoined 5 rounds later; full: not restarted) and a
    half/half partition for 10 rounds.  leave=True: the victims call leave/0
    (psim_leave) at crash_at instead of crashing."""
    sim = make(default_config(n_nodes=n, seed=seed, manager=1, strategy=strategy, fanout=fanout, **cfg))
    rng = np.random.Generator(np.random.PCG64([seed, 7]))
    victims = np.sort(rng.choice(np.arange(1, n, dtype=np.uint32), size=max(1, n // 10),
                                 replace=False)).astype(np.uint32)

    def hook(r):
        if crash_at is not None and r == crash_at:
            (sim.leave if leave else sim.crash)(victims)
        if crash_at is not None and r == crash_at + 5 and strategy != 0:
            sim.join(victims, np.zeros(victims.size, np.uint32))
        if part_at is not None and r == part_at:
            sim.set_partition(W.half_partition(n))
        if part_at is not None and r == part_at + 10:
            sim.clear_partition()
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st


def pl_leave_remote(make, n, seed, rounds, strategy, leave_at=40, k=16, part_at=None, fanout=0):
    """SCAMP with leave/1 (psim_leave_node): a doubling bootstrap, then at
    leave_at k nodes each remove the second entry of their view (the first
    is themselves; full strategy: a random other node); targets distinct.
    Returns (sim, stats, actors, targets)."""
    sim = make(default_config(n_nodes=n, seed=seed, manager=1, strategy=strategy, fanout=fanout))
    rng = np.random.Generator(np.random.PCG64([seed, 9]))
    picked = {}

    def hook(r):
        if r == leave_at:
            v = sim.strategy_nodes()
            actors, targets, used = [], [], set()
            for x in rng.permutation(n):
                if strategy == 0:
                    row = [int(y) for y in rng.permutation(n)[:4] if int(y) != x]
                else:
                    row = [int(y) for y in v["view"][x][: v["view_n"][x]] if int(y) != x]
                if row and row[0] not in used and row[0] not in picked.get("a", []) and x not in used:
                    actors.append(int(x)); targets.append(row[0]); used.update((int(x), row[0]))
                if len(actors) == k:
                    break
            picked["a"], picked["t"] = actors, targets
            sim.leave_node(np.array(actors, np.uint32), np.array(targets, np.uint32))
        if part_at is not None and r == part_at:
            sim.set_partition(W.half_partition(n))
        if part_at is not None and r == part_at + 10:
            sim.clear_partition()
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st, np.array(picked["a"], np.uint32), np.array(picked["t"], np.uint32)


def pl_leave_fixed(make, n, seed, rounds, strategy, leave_at, actors, targets, fanout=0):
    """pl_leave_remote's schedule with the leave/1 pairs given (the pairs a
    run of pl_leave_remote picked): for handles that cannot pick them
    themselves, e.g. RCCL ranks that see only their own rows."""
    sim = make(default_config(n_nodes=n, seed=seed, manager=1, strategy=strategy, fanout=fanout))

    def hook(r):
        if r == leave_at:
            sim.leave_node(np.asarray(actors, np.uint32), np.asarray(targets, np.uint32))
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st


def pl_omission(make, n, seed, rounds, strategy, fanout=0, begin=40, end=60, heal=75, k=None):
    """The crash-fault model's omission faults (prop_partisan_crash_fault_model
    :93-229) on a pluggable handle: a doubling bootstrap; at `begin` k nodes
    start a general omission (begin_omission), k send omissions and k receive
    omissions are installed on pairs drawn from the nodes' views (SCAMP; the
    full strategy: random pairs); at `end` half of each kind ends; at `heal`
    resolve_all_faults_with_heal.  Returns (sim, stats, faults) with faults =
    dict(general=ids, send=(src, dst), recv=(src, dst))."""
    sim = make(default_config(n_nodes=n, seed=seed, manager=1, strategy=strategy, fanout=fanout))
    rng = np.random.Generator(np.random.PCG64([seed, 13]))
    k = k or max(2, n // 32)
    f = {}

    def pairs():
        if strategy == 0:
            s = rng.choice(n, size=k, replace=False).astype(np.uint32)
            d = ((s.astype(np.int64) + 1 + rng.integers(0, n - 1, size=k)) % n).astype(np.uint32)
            return s, d
        v = sim.strategy_nodes()
        src, dst = [], []
        for x in rng.permutation(n):
            row = [int(y) for y in v["view"][x][: v["view_n"][x]] if int(y) != x]
            if row:
                src.append(int(x)); dst.append(row[int(rng.integers(0, len(row)))])
            if len(src) == k:
                break
        return np.array(src, np.uint32), np.array(dst, np.uint32)

    def hook(r):
        if r == begin:
            f["general"] = np.sort(rng.choice(np.arange(1, n), size=k, replace=False)).astype(np.uint32)
            f["send"], f["recv"] = pairs(), pairs()
            sim.begin_omission(f["general"])
            sim.begin_send_omission(*f["send"])
            sim.begin_receive_omission(*f["recv"])
            sim.begin_send_omission(*f["send"])          # a second install keeps one fun
        if r == end:
            h = k // 2
            sim.end_omission(f["general"][:h])
            sim.end_send_omission(f["send"][0][:h], f["send"][1][:h])
            sim.end_receive_omission(f["recv"][0][:h], f["recv"][1][:h])
        if r == heal:
            sim.resolve_all_faults()
    st = sim.run_schedule(W.doubling_join(n, seed), rounds, extra=hook)
    return sim, st, f


def compare_strategy(a, b, full_bits=None):
    """strategy_nodes() of two backends; for the full strategy also the
    member bitsets of the nodes in full_bits"""
    compare_nodes(a.strategy_nodes(), b.strategy_nodes())
    for node in (full_bits or []):
        assert np.array_equal(a.member_bits(node), b.member_bits(node)), node


def compare_stats(a, b):
    assert a.shape == b.shape
    for f in STAT_FIELDS:
        if not np.array_equal(a[f], b[f]):
            bad = np.nonzero((a[f] != b[f]).reshape(len(a), -1).any(1))[0]
            raise AssertionError(f"stats field {f} differs first at round {int(a['round'][bad[0]])}")


def compare_nodes(a, b):
    for f in a.dtype.names:
        if not np.array_equal(a[f], b[f]):
            bad = np.nonzero((a[f] != b[f]).reshape(len(a), -1).any(1))[0]
            raise AssertionError(f"node field {f} differs at nodes {bad[:8].tolist()}")


def active_graph(views):
    return {i: set(int(x) for x in v["act"][: v["act_n"]]) - {i}
            for i, v in enumerate(views) if v["up"]}


def connected(adj):
    if not adj:
        return True
    start = next(iter(adj))
    seen, stack = {start}, [start]
    while stack:
        x = stack.pop()
        for y in adj[x]:
            if y in adj and y not in seen:
                seen.add(y)
                stack.append(y)
    return len(seen) == len(adj)


def asymmetric(adj):
    return [(i, j) for i in adj for j in adj[i] if j in adj and i not in adj[j]]


def random_phash(n, seed):
    """erlang:phash(NodeSpec, 2^32) - 1 per node as an in-BEAM export would
    give it (psim_set_phash_table): random 32-bit values"""
    return np.random.Generator(np.random.PCG64([seed, 0xFA5])).integers(0, 1 << 32, n, dtype=np.uint64).astype(
        np.uint32)


def with_phash(make, seed=7):
    """`make` with a 32-bit phash table installed before the first round."""
    def mk(cfg):
        sim = make(cfg)
        sim.set_phash_table(random_phash(cfg.n_nodes, seed))
        return sim
    return mk


def pl_v1_large_view(make, n=180, seed=29, per_round=20, leave_from=40, leave_to=140, rounds=160):
    """SCAMP v1 with a membership past 80 ids (OTP sets v1 linear hashing,
    SURVEY App. A Q1): every node joins node 0, per_round a round, so node 0
    keeps ~40 % of the N forward_subscriptions (sv1:212-252) and its view
    grows past 80 (expansions at 81, 86, ...); from leave_from node 0
    removes one member a round with leave/1 (sv1:102-122: sets:del_element)
    until its view drops below 3 n (contractions).  The leave targets are
    read from the handle's own view."""
    sim = make(default_config(n_nodes=n, seed=seed, manager=1, strategy=1))
    sched = [(0, np.array([0], np.uint32), np.array([W.NONE], np.uint32))]
    for r, lo in enumerate(range(1, n, per_round), start=1):
        ids = np.arange(lo, min(n, lo + per_round), dtype=np.uint32)
        sched.append((r, ids, np.zeros(ids.size, np.uint32)))
    trace = []

    def hook(r):
        v = sim.strategy_nodes(0, 1)[0]
        trace.append((int(v["view_n"]), int(v["view_slots"])))
        if leave_from <= r < leave_to and v["up"]:
            row = [int(x) for x in v["view"][: v["view_n"]] if int(x) != 0]
            if row:
                sim.leave_node(np.array([0], np.uint32), np.array([row[len(row) // 2]], np.uint32))
    st = sim.run_schedule(sched, rounds, extra=hook)
    return sim, st, trace
