"""Config E per-round attribution (diagnostic): bench.py's exact E schedule
(doubling bootstrap, settle, broadcast every 10 rounds, 20 % churn from
round STEADY_ROUNDS over 100 rounds, the half/half partition 20 rounds into
the window), with PSIM_PHASE_TIMERS=1 so every phase of a round is timed by
HIP events.  Prints, per round of the last --rounds rounds, the host wall
time of psim_step, each phase's device time and the remainder (host time
between phases: syncs, uploads, allocations).
Usage: PSIM_PHASE_TIMERS=1 python profiles/e_attrib.py [--nodes N] [--warmup 5] [--steps 60]"""
import argparse
import os
import sys
import time

os.environ.setdefault("PSIM_PHASE_TIMERS", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from partisan_amd import Simulator, workloads as W  # noqa: E402
from partisan_amd.sim import default_config  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--nodes", type=int, default=1 << 23)
p.add_argument("--warmup", type=int, default=5)
p.add_argument("--steps", type=int, default=60)
p.add_argument("--settle", type=int, default=60)
p.add_argument("--seed", type=int, default=1)
a = p.parse_args()
n = a.nodes
STEADY, BP = 40, 10
t0 = time.perf_counter()
sim = Simulator(default_config(n_nodes=n, seed=a.seed))
boot = W.doubling_join(n, a.seed)
sim.run_schedule(boot, boot[-1][0] + 1 + a.settle)
print(f"setup {time.perf_counter() - t0:.1f} s, round {sim.round}", flush=True)
churn = {r: (v, c) for r, v, c in W.churn_schedule(n, a.seed, 0.2, STEADY, 100)}
part = W.half_partition(n)
t_start = STEADY + a.warmup
p_on, p_off = t_start + 20, t_start + 40
tot = {}
rows = 0
for i in range(t_start + a.steps):
    ev = []
    if i % BP == 0:
        sim.broadcast(0, (i // BP) % 0x10000)
        ev.append("B")
    if i in churn:
        sim.crash(churn[i][0])
        ev.append("C")
    if i - 1 in churn:
        sim.join(churn[i - 1][0], churn[i - 1][1])
        ev.append("J")
    if i == p_on:
        sim.set_partition(part)
        ev.append("P")
    if i == p_off:
        sim.clear_partition()
        ev.append("H")
    t1 = time.perf_counter()
    st = sim.step(1)[0]
    wall = (time.perf_counter() - t1) * 1e3
    kt = {k: v[0] for k, v in sim.kernel_times().items() if v[1]}
    dev = sum(kt.values())
    if i >= t_start:
        rows += 1
        for k, v in kt.items():
            tot[k] = tot.get(k, 0.0) + v
        tot["wall"] = tot.get("wall", 0.0) + wall
        tot["host"] = tot.get("host", 0.0) + wall - dev
    print(f"r{i:3d} {''.join(ev):4s} wall {wall:8.2f} " + " ".join(f"{k} {v:7.2f}" for k, v in kt.items())
          + f" host {wall - dev:7.2f} | proc {int(st['nodes_processed'])} emit {int(st['emitted'].sum())}",
          flush=True)
print("avg over the window (ms/round): " + " ".join(f"{k} {v / max(1, rows):.2f}" for k, v in tot.items()), flush=True)
sim.close()
