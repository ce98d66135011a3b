"""Reference parity through the in-BEAM harness (erlang/harness/README.md).

  python erlang/harness/compare_trace.py scenario config_a DIR [BUCKETS]
      writes DIR/config_a.terms (the event script psim_harness:run/2 -- or,
      for the *_pl scenarios, psim_strategy_harness:run/2 -- reads)
      and DIR/config_a.oracle (the CPU oracle's record stream of the same
      scenario: one line per emitted message, in the harness's format; its
      first line `S config_a` names the scenario).  With BUCKETS (a file of
      `B id hash` or `id hash` lines) the oracle orders views by that
      sets v1 table (psim_set_phash_table) instead of its stand-in.
  python erlang/harness/compare_trace.py compare DIR/config_a.harness DIR/config_a.oracle
      diffs the two streams round by round; exit status 1 at the first
      differing record.  The harness writes the real view order -- a line
      `B id hash` per node, hash = erlang:phash(NodeSpec, 2^32) - 1 (App.
      A Q1) -- which compare copies to DIR/bucket16.txt and, when it differs
      from the table the oracle stream was made with, uses to regenerate that
      stream (DIR/config_a.oracle_b) before diffing: one harness run is a
      complete comparison.

The oracle is the checker (test infrastructure); the GPU engine is pinned to
it bit for bit by tests/test_gpu_parity.py, so harness == oracle extends to
harness == engine."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from partisan_amd import _abi  # noqa: E402
from partisan_amd import workloads as W  # noqa: E402
from partisan_amd.sim import default_config  # noqa: E402

NONE = 0xFFFFFFFF

SCENARIOS = {
    # config A (test/partisan_SUITE.erl:1591-1601): node i joins node 0 at
    # round i, 200 rounds, a broadcast from node 0 at round 200, 40 more
    "config_a": dict(n=32, seed=1, rounds=240, joins=lambda n, s: W.sequential_join(n),
                     bcast=[(200, 0, 7)], crash={}),
    # a doubling bootstrap with crashes (EXIT handling) and broadcasts
    "doubling_crash_256": dict(n=256, seed=3, rounds=80, joins=lambda n, s: W.doubling_join(n, s),
                               bcast=[(30, 0, 1), (60, 0, 2)], crash={40: list(range(5, 256, 17))}),
    # the pluggable manager's strategies (erlang/harness/psim_strategy_harness.erl;
    # pl:384, :881-903, :986-1044, :1153-1195): configs B and D in miniature,
    # reference semantics (fanout 0), with crashes, a partition and leave/1
    "full_16_pl": dict(n=16, seed=11, rounds=80, joins=lambda n, s: W.doubling_join(n, s), bcast=[],
                       crash={40: [5]}, strategy="full"),
    "scamp_v1_128_pl": dict(n=128, seed=11, rounds=100, joins=lambda n, s: W.doubling_join(n, s), bcast=[],
                            crash={40: [3, 77]}, part=(60, 70), leave={50: [(9, 10)]}, strategy="scamp_v1"),
    "scamp_v2_128_pl": dict(n=128, seed=11, rounds=100, joins=lambda n, s: W.doubling_join(n, s), bcast=[],
                            crash={40: [3, 77]}, part=(60, 70), leave={50: [(9, 10)]}, strategy="scamp_v2"),
}
STRATEGIES = {"full": 0, "scamp_v1": 1, "scamp_v2": 2}


def read_buckets(path, n=None):
    """`B id hash` (harness output: erlang:phash(NodeSpec, 2^32) - 1) or
    `id hash` lines -> uint32 table; a 16-slot bucket table (0..15) reads
    the same way (psim_set_phash_table takes it as a hash with zero high bits)"""
    rows = []
    for l in open(path):
        f = l.split()
        if f and f[0] == "B":
            f = f[1:]
        if len(f) == 2:
            rows.append((int(f[0]), int(f[1])))
    m = n if n is not None else (max(i for i, _ in rows) + 1 if rows else 0)
    tab = np.zeros(m, np.uint32)
    seen = np.zeros(m, bool)
    for i, b in rows:
        if i < m:
            tab[i], seen[i] = b, True
    if not seen.all():
        raise ValueError(f"{path}: not a hash table of {m} nodes")
    return tab


def scenario(name, out_dir, buckets=None):
    sc = SCENARIOS[name]
    n, seed, rounds = sc["n"], sc["seed"], sc["rounds"]
    joins = sc["joins"](n, seed)
    strategy = sc.get("strategy")
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, name + ".terms"), "w") as f:
        extra = f", strategy => {strategy}, periodic_interval => 10, scamp_c => 5" if strategy else ""
        f.write(f"{{config, #{{n_nodes => {n}, seed => {seed}, rounds => {rounds}{extra}}}}}.\n")
        for r, ids, contacts in joins:
            pairs = ", ".join(f"{{{int(i)}, {'none' if int(c) == NONE else int(c)}}}" for i, c in zip(ids, contacts))
            f.write(f"{{join, {r}, [{pairs}]}}.\n")
        for r, ids in sc["crash"].items():
            f.write(f"{{crash, {r}, [{', '.join(str(i) for i in ids)}]}}.\n")
        for r, root, msg in sc["bcast"]:
            f.write(f"{{broadcast, {r}, {root}, {msg}}}.\n")
        if "part" in sc:
            g = ", ".join(str(int(x)) for x in W.half_partition(n))
            f.write(f"{{partition, {sc['part'][0]}, [{g}]}}.\n{{clear_partition, {sc['part'][1]}}}.\n")
        for r, pairs in sc.get("leave", {}).items():
            f.write(f"{{leave, {r}, [{', '.join(f'{{{a}, {t}}}' for a, t in pairs)}]}}.\n")
    tab = read_buckets(buckets, n) if buckets else None
    write_stream(name, os.path.join(out_dir, name + ".oracle"), tab)
    print(f"wrote {name}.terms and {name}.oracle")


def write_stream(name, path, tab=None):
    sc = SCENARIOS[name]
    n, seed, rounds = sc["n"], sc["seed"], sc["rounds"]
    lines = oracle_stream(n, seed, rounds, sc["joins"](n, seed), sc["bcast"], sc["crash"],
                          strategy=sc.get("strategy"), part=sc.get("part"), leave=sc.get("leave", {}),
                          buckets=tab)
    with open(path, "w") as f:
        f.write(f"S {name}\n")
        if tab is not None:
            f.write("".join(f"B {i} {int(b)}\n" for i, b in enumerate(tab)))
        f.write("\n".join(lines) + "\n")
    return len(lines)


def oracle_stream(n, seed, rounds, joins, bcast, crash, strategy=None, part=None, leave=None, buckets=None):
    from _oracle import Oracle
    if strategy:
        o = Oracle(default_config(n_nodes=n, seed=seed, manager=_abi.MANAGER_PLUGGABLE,
                                  strategy=STRATEGIES[strategy], fanout=0, scamp_c=5, periodic_interval=10))
    else:
        o = Oracle(default_config(n_nodes=n, seed=seed))
    if buckets is not None:
        o.set_phash_table(buckets)
    lib = o._lib
    ev = {}
    for r, ids, contacts in joins:
        ev.setdefault(r, []).append((ids, contacts))
    bc = {r: (root, msg) for r, root, msg in bcast}
    lines = []
    for r in range(rounds):
        for ids, contacts in ev.get(r, []):
            o.join(ids, contacts)
        if r in crash:
            o.crash(np.array(crash[r], np.uint32))
        if r in bc:
            o.broadcast(*bc[r])
        if part and r == part[0]:
            o.set_partition(W.half_partition(n))
        if part and r == part[1]:
            o.clear_partition()
        if leave and r in leave:
            o.leave_node([a for a, _ in leave[r]], [t for _, t in leave[r]])
        st = np.zeros(1, _abi.STATS_DTYPE)
        assert lib.orc_round_emit(o._h, st.ctypes.data) == 0
        k = C.c_size_t()
        lib.orc_get_outbox(o._h, None, 0, C.byref(k))
        box = np.zeros((k.value, 16), np.uint32)
        lib.orc_get_outbox(o._h, box.ctypes.data, k.value, C.byref(k))
        for rec in box:
            dst, src, seq, tt = (int(x) for x in rec[:4])
            t, ttl, nex = tt & 0xFF, (tt >> 8) & 0xFF, (tt >> 16) & 0xFF
            ex = "".join(f" {int(x)}" for x in rec[8:8 + nex])
            lines.append(f"R {r} {src} {seq} {dst} {t} {ttl} {int(rec[4])} {int(rec[5])} {int(rec[6])} {nex}{ex}")
        box = np.ascontiguousarray(box)
        assert lib.orc_round_absorb(o._h, box.ctypes.data, box.shape[0]) == 0
    return lines


def compare(harness, oracle):
    h = [l.rstrip("\n") for l in open(harness) if l.startswith("R ")]
    o = [l.rstrip("\n") for l in open(oracle) if l.startswith("R ")]
    buckets = [l for l in open(harness) if l.startswith("B ")]
    if buckets:
        path = os.path.join(os.path.dirname(os.path.abspath(harness)), "bucket16.txt")
        with open(path, "w") as f:
            f.writelines(buckets)
        names = [l.split()[1] for l in open(oracle) if l.startswith("S ")]
        used = [l for l in open(oracle) if l.startswith("B ")]
        if names and names[0] in SCENARIOS and sorted(used) != sorted(buckets):
            # the stream was made with another view order: remake it with the
            # harness's erlang:phash table, then diff against that
            tab = read_buckets(path, SCENARIOS[names[0]]["n"])
            regen = os.path.splitext(oracle)[0] + ".oracle_b"
            write_stream(names[0], regen, tab)
            print(f"oracle stream regenerated with the harness's bucket table: {regen}")
            o = [l.rstrip("\n") for l in open(regen) if l.startswith("R ")]
    for i, (a, b) in enumerate(zip(h, o)):
        if a != b:
            print(f"record {i} differs:\n  harness {a}\n  oracle  {b}")
            return 1
    if len(h) != len(o):
        print(f"record counts differ: harness {len(h)}, oracle {len(o)}")
        return 1
    print(f"{len(h)} records identical")
    return 0


if __name__ == "__main__":
    if sys.argv[1] == "scenario":
        scenario(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
