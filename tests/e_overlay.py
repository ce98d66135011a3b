"""The overlay after config E's churn: components and
reliability once churn has ended, and a classification of the live nodes
outside the giant component.

Config E (bench.py --workload E, partisan_amd.workloads.BenchSchedule):
doubling bootstrap, 0.2 N crashes over phase rounds 40-139 (each victim
restarts and rejoins a random live node the next round), a half/half
partition for 20 rounds of the window, a broadcast from node 0 every 10
rounds.  At each report point this records, over the live nodes:
  components / giant   weakly connected components over active links
                       (checked against psim_get_histograms)
  outside              live nodes outside the giant component, split into
    isolated_restart   empty active view, (re)started in the last 20 rounds
    isolated_old       empty active view, up for longer
    small_comp         in a component of >= 2 nodes that is not the giant one
    outside_victims    ... churn victims (crashed, restarted, rejoined)
    outside_lost_join  ... victims whose rejoin crossed the partition while
                       it was on: the JOIN is dropped, the restarted node's
                       views stay empty and HyParView never retries it
  delivered            live nodes holding the tracked (latest) broadcast
and, after the last point, one more broadcast with no further events:
  delivered_10/20/40   the fraction of live nodes holding it 10, 20, 40
                       rounds on; last_round / hops of its last delivery
Report points are phase rounds after the last churn join (round 140):
+9 (round 2 took its E numbers near +5), +49 and +89 (>= 40 settle rounds):
nine rounds after a broadcast, so the tracked one has run its course.

Usage (GPU box):  python tests/e_overlay.py --backend gpu --nodes 65536 1048576 4194304
       (CPU here): python tests/e_overlay.py --backend oracle --nodes 16384 65536
Writes one JSON line per (backend, n) to stdout.  The oracle is the checker
(tests/ only); the same seeds give bit-identical runs on both backends."""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]

from partisan_amd import workloads as W  # noqa: E402
from partisan_amd.sim import default_config  # noqa: E402

CHURN_END = W.BenchSchedule.STEADY_ROUNDS + 100     # phase round of the last churn join
POINTS = (9, 49, 89)
CHUNK = 1 << 17


def lost_joins(sched):
    """(victims, lost): masks over the nodes -- churn victims, and victims
    whose last rejoin went to a contact across the half/half partition while
    it was on (a JOIN sent in round p_on - 1 arrives partitioned)"""
    victims = np.zeros(sched.n, bool)
    lost = np.zeros(sched.n, bool)
    last = {}
    for r, (v, c) in sorted(sched.churn.items()):
        victims[v] = True
        for a, b in zip(v.tolist(), c.tolist()):
            last[a] = (r + 1, b)                  # rejoins the round after its crash
    for a, (j, b) in last.items():
        lost[a] = sched.p_on - 1 <= j < sched.p_off and sched.part[a] != sched.part[b]
    return victims, lost


def classify(sim, sched=None, recent=20):
    """The overlay's components over the live nodes' active links, and the
    classification of the live nodes outside the giant component."""
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    n = sim.n
    up = np.zeros(n, bool)
    start = np.zeros(n, np.int64)
    act_n = np.zeros(n, np.int64)
    src, dst = [], []
    for f in range(0, n, CHUNK):
        v = sim.nodes(f, min(CHUNK, n - f))
        k = np.arange(f, f + len(v))
        up[k] = v["up"] != 0
        start[k] = v["start_round"]
        act_n[k] = v["act_n"]
        a = v["act"].astype(np.int64)
        col = np.arange(a.shape[1])[None, :]
        m = (col < v["act_n"][:, None]) & (a != k[:, None]) & (v["up"][:, None] != 0)
        src.append(np.broadcast_to(k[:, None], a.shape)[m])
        dst.append(a[m])
    src, dst = np.concatenate(src), np.concatenate(dst)
    keep = up[dst]
    src, dst = src[keep], dst[keep]
    g = coo_matrix((np.ones(src.size, np.int8), (src, dst)), shape=(n, n))
    _, lab = connected_components(g, directed=True, connection="weak")
    live = np.flatnonzero(up)
    sizes = np.bincount(lab[live], minlength=lab.max() + 1)
    giant = int(np.argmax(sizes))
    out = live[lab[live] != giant]
    rnd = sim.round
    isolated = act_n[out] <= 1                    # (the view holds self)
    restart = start[out] + recent >= rnd
    extra = {}
    if sched is not None:
        victims, lost = lost_joins(sched)
        extra = {"outside_victims": int(victims[out].sum()), "outside_lost_join": int(lost[out].sum()),
                 "lost_joins": int(lost.sum())}
    h = sim.histograms()
    comps = int((sizes > 0).sum())
    assert comps == h["components"] and int(sizes[giant]) == h["largest_component"], \
        (comps, h["components"], int(sizes[giant]), h["largest_component"])
    return {"round": int(rnd), "n_up": int(live.size), "components": comps, "giant": int(sizes[giant]),
            "outside": int(out.size), "outside_frac": out.size / max(live.size, 1),
            "isolated_restart": int((isolated & restart).sum()), "isolated_old": int((isolated & ~restart).sum()),
            "small_comp": int((~isolated).sum()), "small_comp_max": int(np.sort(sizes)[-2]) if comps > 1 else 0,
            "delivered": int(h["delivered"]), "delivered_frac": h["delivered"] / max(live.size, 1)} | extra


def reliability(sim, sched, i, marks=(10, 20, 40)):
    """One more broadcast from node 0 at phase round i (a broadcast round),
    then no further events: live nodes holding it after each mark."""
    assert sched.bcast_round(i)
    sched.apply(sim, i)
    out, done = {}, 0
    for m in marks:
        sim.step(m - done)
        done = m
        h = sim.histograms()
        out[f"delivered_{m}"] = h["delivered"] / max(h["n_up"], 1)
    out["last_round"] = int(h["last_round"])
    out["hops"] = int(np.flatnonzero(h["hop"])[-1]) if h["hop"].any() else 0
    return out


def run(make, n, seed=1, warmup=10, points=POINTS, schedule="doubling"):
    sched = W.BenchSchedule("E", schedule, n, seed, warmup)
    sim = make(default_config(n_nodes=n, seed=seed))
    boot, until = sched.bootstrap()
    sim.run_schedule(boot, until)
    want = {CHURN_END + p for p in points}
    rows = []
    i = 0
    while want:
        sched.apply(sim, i)
        k = 1
        while i + k not in want and not sched.has_events(i + k):
            k += 1
        sim.step(k)
        i += k
        if i in want:
            want.discard(i)
            rows.append({"after_churn": i - CHURN_END} | classify(sim, sched))
    return rows, reliability(sim, sched, i + 1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--backend", choices=["gpu", "oracle"], required=True)
    p.add_argument("--nodes", type=int, nargs="+", required=True)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--schedule", choices=["doubling", "survey"], default="doubling")
    a = p.parse_args()
    if a.backend == "gpu":
        from partisan_amd import Simulator as make
    else:
        from _oracle import Oracle as make
    for n in a.nodes:
        t = time.time()
        rows, rel = run(make, n, a.seed, schedule=a.schedule)
        print(json.dumps({"backend": a.backend, "nodes": n, "seed": a.seed, "schedule": a.schedule,
                          "wall_s": round(time.time() - t, 1),
                          "points": rows, "reliability": rel}), flush=True)


if __name__ == "__main__":
    main()
