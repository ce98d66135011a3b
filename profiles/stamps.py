"""Per-phase cycle breakdown of k_consume (diagnostic builds, -DPSIM_STAMPS).

Runs config C like bench.py and prints the summed s_memtime deltas per phase
of the wave-per-node consume kernel over the timed rounds.
Usage: python profiles/stamps.py [--nodes N] [--steps K]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = {0: "idle-node", 1: "setup+loads", 2: "join+exits", 3: "inbox-chunk/misc",
         13: "promotion", 14: "shuffle", 15: "notify-replay", 21: "origin",
         22: "lazy-tick", 23: "writeback", 24: "loop", 25: "shuffle:forward",
         26: "shuffle:accept-sublist", 27: "shuffle:accept-reply", 28: "shuffle:accept-merge",
         29: "k_pt setup/inbox-misc", 30: "k_pt writeback", 31: "k_pt loop"}
HV = ["JOIN", "FWD_JOIN", "NEIGHBOR", "DISCONNECT", "NEIGHBOR_REQ", "NEIGHBOR_ACC",
      "NEIGHBOR_REJ", "SHUFFLE", "SHUFFLE_REPLY"]
PT = ["BROADCAST", "PRUNE", "IHAVE", "IGNORED_IHAVE", "GRAFT"]
for i, n in enumerate(HV):
    NAMES[4 + i] = "hv:" + n
for i, n in enumerate(PT):
    NAMES[16 + i] = "pt:" + n


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--nodes", type=int, default=1 << 20)
    p.add_argument("--steps", type=int, default=20)
    a = p.parse_args()
    from partisan_amd import Simulator, _lib
    from partisan_amd import workloads as W
    from partisan_amd.sim import default_config

    lib = _lib.load()
    lib.psim_debug_stamps.restype = C.c_int
    lib.psim_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * 32)()
    sim = Simulator(default_config(n_nodes=a.nodes, seed=1))
    boot = W.doubling_join(a.nodes, 1)
    sim.run_schedule(boot, boot[-1][0] + 61)
    # bench.py's schedule: 45 untimed broadcast rounds (steady state), then
    # the measured rounds, a broadcast from node 0 every 10 rounds
    k = 0
    for i in range(45):
        if i % 10 == 0:
            sim.broadcast(0, k)
            k += 1
        sim.step(1)
    if lib.psim_debug_stamps(buf, 32) != 32:
        print("library built without -DPSIM_STAMPS")
        return
    st = []
    for i in range(45, 45 + a.steps):
        if i % 10 == 0:
            sim.broadcast(0, k)
            k += 1
        st.append(sim.step(1))
    lib.psim_debug_stamps(buf, 32)
    st = np.concatenate(st)
    v = np.array(buf[:], np.float64)
    tot = v.sum()
    print(f"rounds {a.steps}  processed {int(st['nodes_processed'].sum())}  "
          f"delivered {int(st['delivered'].sum())}  emitted {int(st['emitted'].sum())}")
    print(f"total wave-ticks {tot:.4g} (s_memtime: shader clock)")
    dl = st["delivered"].sum(axis=0) / a.steps
    print("delivered/round: " + ", ".join(f"{n}={int(dl[i])}" for i, n in enumerate(HV + PT) if dl[i]))
    for k in np.argsort(-v):
        if v[k] == 0:
            continue
        print(f"  {NAMES.get(int(k), str(k)):18s} {v[k] / tot * 100:6.2f}%  {v[k] / a.steps:.4g}/round")


if __name__ == "__main__":
    main()
