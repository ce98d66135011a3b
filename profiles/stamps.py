"""Per-phase cycle breakdown of the wave-per-node kernels (diagnostic
builds, -DPSIM_STAMPS: `make -C partisan_amd/csrc stamps`, loaded with
PSIM_LIB=stamps).

Runs bench.py's config C schedule (workloads.BenchSchedule, survey by
default) and prints the summed s_memtime deltas per phase of k_consume /
k_pt and of k_consume_lite over the timed rounds.
Usage: PSIM_LIB=stamps python profiles/stamps.py [--nodes N] [--steps K] [--schedule survey|doubling]
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
HALF = {8: "loop / wait for the node's loads", 0: "begin + connection cache", 6: "inbox record parse",
        1: "SHUFFLE relay", 2: "terminal: sublist", 3: "terminal: reply send", 4: "merge_exchange",
        5: "shuffle start", 7: "writeback + flush", 9: "body's end (the other half's work)"}
PTL = {0: "list entry, rows, records, preconditions", 1: "k_pt list append", 2: "active row + connection mask",
       3: "sets / table loads", 4: "update_peers (every message)", 5: "BROADCAST first: eager push + lazy adds",
       9: "IGNORED_IHAVE ack", 10: "answer send",
       11: "handler loop control", 12: "lazy tick", 13: "writeback", 14: "kernel end"}
LITE = {0: "wait for the node's loads", 1: "begin_node", 2: "inbox chunk / record parse", 3: "SHUFFLE_REPLY merge",
        4: "SHUFFLE relay", 5: "terminal: sublist", 6: "terminal: reply send", 7: "terminal: merge",
        8: "shuffle start", 9: "next node's 2nd-stage loads", 10: "writeback", 11: "next node's loads"}


def table(v, names, steps):
    tot = v.sum()
    if tot == 0:
        return
    print(f"  total wave-ticks {tot:.4g} ({tot / steps:.4g}/round)")
    for k in np.argsort(-v):
        if v[k]:
            print(f"    {names.get(int(k), str(k)):30s} {v[k] / tot * 100:6.2f}%  {v[k] / steps:.4g}/round")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--nodes", type=int, default=1 << 20)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--schedule", default="survey")
    p.add_argument("--workload", default="C", choices=("C", "E"))
    a = p.parse_args()
    from partisan_amd import Simulator, _lib
    from partisan_amd import workloads as W
    from partisan_amd.sim import default_config

    lib = _lib.load()
    lib.psim_debug_stamps.restype = C.c_int
    lib.psim_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * 96)()
    sim = Simulator(default_config(n_nodes=a.nodes, seed=1))
    sched = W.BenchSchedule(a.workload, a.schedule, a.nodes, 1, a.warmup)
    boot, until = sched.bootstrap()
    sim.run_schedule(boot, until)
    for i in range(sched.t_start):
        sched.apply(sim, i)
        sim.step(1)
    if lib.psim_debug_stamps(buf, 96) != 96:
        print("library built without -DPSIM_STAMPS (make -C partisan_amd/csrc stamps; PSIM_LIB=stamps)")
        return
    st = []
    for i in range(sched.t_start, sched.t_start + a.steps):
        sched.apply(sim, i)
        st.append(sim.step(1))
    lib.psim_debug_stamps(buf, 96)
    st = np.concatenate(st)
    v = np.array(buf[:], np.float64)
    print(f"{a.workload}, {a.schedule} schedule, {a.nodes} nodes, rounds {a.steps}: processed {int(st['nodes_processed'].sum())} "
          f"delivered {int(st['delivered'].sum())} emitted {int(st['emitted'].sum())} (s_memtime ticks)")
    dl = st["delivered"].sum(axis=0) / a.steps
    print("delivered/round: " + ", ".join(f"{n}={int(dl[i])}" for i, n in enumerate(HV + PT) if dl[i]))
    print("k_consume / k_pt:")
    table(v[:32], NAMES, a.steps)
    if v[32:48].any():
        print("k_consume_lite:")
        table(v[32:48], LITE, a.steps)
    if v[48:64].any():
        print("k_ptl (wave time by phase; a divergent handler's branches each charged their own):")
        table(v[48:64], PTL, a.steps)
    if v[64:].any():
        print("k_lite_half (each half's phases; both halves summed):")
        table(v[64:80] + v[80:96], HALF, a.steps)


if __name__ == "__main__":
    main()
