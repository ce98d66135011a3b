"""Per-round wall time of config E (diagnostic): which rounds are slow.
Usage: python profiles/e_steps.py [--nodes N] [--rounds R]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from partisan_amd import Simulator, workloads as W  # noqa: E402
from partisan_amd.sim import default_config  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--nodes", type=int, default=1 << 23)
p.add_argument("--rounds", type=int, default=70)
a = p.parse_args()
n = a.nodes
sim = Simulator(default_config(n_nodes=n, seed=1))
boot = W.doubling_join(n, 1)
sim.run_schedule(boot, boot[-1][0] + 61)
churn = {r: (v, c) for r, v, c in W.churn_schedule(n, 1, 0.2, 0, 100)}
part = W.half_partition(n)
for i in range(a.rounds):
    if i % 10 == 0:
        sim.broadcast(0, i // 10)
    if i in churn:
        sim.crash(churn[i][0])
    if i - 1 in churn:
        sim.join(churn[i - 1][0], churn[i - 1][1])
    if i == 20:
        sim.set_partition(part)
    if i == 40:
        sim.clear_partition()
    t0 = time.perf_counter()
    st = sim.step(1)[0]
    dt = (time.perf_counter() - t0) * 1e3
    kt = sim.kernel_times()
    print(f"round {i:3d} {dt:8.2f} ms  consume {kt['consume'][0]:7.2f}  proc {int(st['nodes_processed'])} "
          f"deliv {int(st['delivered'].sum())} emit {int(st['emitted'].sum())} ovf {int(st['overflow'])}", flush=True)
