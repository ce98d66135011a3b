"""The headline overlay's disconnected nodes: config C on
the survey schedule (bench.py's default line, partisan_amd.workloads
BenchSchedule "C"/"survey") ends with a few small components beside the
giant one -- 16 components, 902 nodes outside at 2^20.  This classifies them
at report points through the run:

  components / giant / outside   weakly connected components over active links
  isolated            live nodes with an empty active view (a lost or evicted
                      JOIN leaves one: hv:500-515 sends it once)
  small_comp          nodes in components of >= 2 nodes that are not the giant
  min_peers_outside   the fewest active peers any outside node holds
  comp_sizes          the small components' sizes
  pas_into_giant      mean passive-view entries of an outside node that lie in
                      the giant component
  stable_since        the first report point from which the outside set is the
                      same set of nodes as at the end

The finding: no outside node is isolated.  Each sits in
a closed component of >= 2 nodes that formed during the join ramp, when
eviction DISCONNECTs (add_to_active_view on a full view, hv:1371-1386,
:1467-1510) cut its last links to the rest.  With >= 2 active peers (all of
them at 2^18 and 2^20) a node is at min_active_size (3 with the node
itself), so random_promotion (hv:542-556, has_reached_the_limit) never
fires; with 1 (a few at 2^24) its low-priority NEIGHBOR requests meet full
views; shuffles walk only the component's own active links, and the passive
view is promoted only on a failure.  Nothing in the protocol merges such a
component again; the oracle (the reference's handlers) shows the same
components, and the GPU equals it bit for bit (test_bench_schedule_parity
at 2^20).

Usage (GPU box):  python tests/c_overlay.py --backend gpu --nodes 262144 1048576
       (CPU here): python tests/c_overlay.py --backend oracle --nodes 16384 65536
One JSON line per (backend, n)."""
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

CHUNK = 1 << 17
# report points: rounds of the bootstrap (the ramp ends at 64), then the end
# of the bench's window (warmup 5 + 20 timed rounds + 5)
POINTS = (48, 64, 72, 80, 96, 132, W.SURVEY_RAMP + W.BenchSchedule.SURVEY_WARM)
WARMUP, WINDOW = 5, 25


def classify(sim):
    """components over the live nodes' active links, and the outside nodes"""
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    n = sim.n
    up = np.zeros(n, bool)
    act_n = np.zeros(n, np.int64)
    pas_rows, pas_n = [], np.zeros(n, np.int64)
    src, dst = [], []
    for f in range(0, n, CHUNK):
        v = sim.nodes(f, min(CHUNK, n - f))
        k = np.arange(f, f + len(v))
        up[k] = v["up"] != 0
        act_n[k] = v["act_n"]
        pas_n[k] = v["pas_n"]
        pas_rows.append(v["pas"].astype(np.int64))
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
    peers = act_n[out] - 1                        # (the view holds the node itself)
    pas = np.concatenate(pas_rows)[out]
    pm = np.arange(pas.shape[1])[None, :] < pas_n[out][:, None]
    into = ((lab[np.where(pm, pas, 0)] == giant) & pm).sum(axis=1)
    small = np.sort(sizes[(sizes > 0) & (np.arange(sizes.size) != giant)])
    return {"round": int(sim.round), "n_up": int(live.size), "components": int((sizes > 0).sum()),
            "giant": int(sizes[giant]), "outside": int(out.size), "outside_frac": out.size / max(live.size, 1),
            "isolated": int((peers <= 0).sum()), "small_comp": int((peers > 0).sum()),
            "min_peers_outside": int(peers.min()) if out.size else None,
            "comp_sizes": small.tolist()[-24:],
            "pas_into_giant": float(into.mean()) if out.size else None}, set(out.tolist())


def run(make, n, seed=1, points=POINTS):
    sched = W.BenchSchedule("C", "survey", n, seed, WARMUP)
    sim = make(default_config(n_nodes=n, seed=seed))
    boot, until = sched.bootstrap()
    rows, sets = [], []
    for p in points:
        sim.run_schedule(boot, p)
        r, s = classify(sim)
        rows.append(r)
        sets.append(s)
    sim.run_schedule(boot, until)
    for i in range(sched.t_start + WINDOW):
        sched.apply(sim, i)
        sim.step(1)
    r, s = classify(sim)
    h = sim.histograms()
    assert r["components"] == h["components"] and r["giant"] == h["largest_component"], (r, h["components"])
    r["delivered_frac"] = h["delivered"] / max(h["n_up"], 1)
    rows.append(r)
    sets.append(s)
    stable = next(rows[k]["round"] for k in range(len(sets)) if all(sets[j] == s for j in range(k, len(sets))))
    if not points:
        stable = None                             # (no earlier report point to compare with)
    return {"rows": rows, "stable_since": stable}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--backend", choices=["gpu", "oracle"], required=True)
    p.add_argument("--nodes", type=int, nargs="+", required=True)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--points", type=int, nargs="*", default=list(POINTS),
                   help="bootstrap rounds to classify at before the window's end (none: the end only)")
    a = p.parse_args()
    if a.backend == "gpu":
        from partisan_amd import Simulator as make
    else:
        from _oracle import Oracle as make
    for n in a.nodes:
        t = time.time()
        r = run(make, n, a.seed, tuple(a.points))
        print(json.dumps({"backend": a.backend, "nodes": n, "seed": a.seed, "wall_s": round(time.time() - t, 1)} | r),
              flush=True)


if __name__ == "__main__":
    main()
