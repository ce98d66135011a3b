"""Diagnostic: which nodes fill their disconnect-id maps under config E.
Runs bench.py's E schedule (doubling bootstrap, settle, churn + partition,
broadcasts every 10 rounds) at N nodes and reports the overflow by round
phase and the nodes whose sent / recv maps are full.
Usage: python profiles/diag/idmap_full.py N [rounds_after_settle]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT]
from partisan_amd import Simulator, workloads as W  # noqa: E402
from partisan_amd.sim import default_config  # noqa: E402

n = int(sys.argv[1])
after = int(sys.argv[2]) if len(sys.argv) > 2 else 145
sim = Simulator(default_config(n_nodes=n, seed=1))
boot = W.doubling_join(n, 1)
st = sim.run_schedule(boot, boot[-1][0] + 61)
print("bootstrap+settle rounds", len(st), "overflow by kind", st["overflow_by"].sum(0).tolist(), flush=True)
churn = {r: (v, c) for r, v, c in W.churn_schedule(n, 1, 0.2, 40, 100)}
part = W.half_partition(n)
ovf = []
for i in range(after):
    if i % 10 == 0:
        sim.broadcast(0, i // 10)
    if i in churn:
        sim.crash(churn[i][0])
    if i - 1 in churn:
        sim.join(churn[i - 1][0], churn[i - 1][1])
    if i == 65:
        sim.set_partition(part)
    if i == 85:
        sim.clear_partition()
    s = sim.step(1)
    ovf.append(s["overflow_by"][0].tolist())
ovf = np.array(ovf)
print("overflow by round (kind 0 idmap):", {i: int(v) for i, v in enumerate(ovf[:, 0]) if v})
full_s, full_r, top = [], [], []
step = 1 << 16
for lo in range(0, n, step):
    v = sim.nodes(lo, min(step, n - lo))
    fs = np.nonzero(v["sent_n"] >= 64)[0]
    fr = np.nonzero(v["recv_n"] >= 64)[0]
    full_s += (fs + lo).tolist()
    full_r += (fr + lo).tolist()
    for j in set(fs.tolist()) | set(fr.tolist()):
        top.append((lo + j, int(v["sent_n"][j]), int(v["recv_n"][j]), int(v["epoch"][j]), int(v["up"][j]),
                    int(v["act_n"][j]), int(v["pas_n"][j])))
print("full sent maps", len(full_s), "full recv maps", len(full_r))
print("examples (id, sent_n, recv_n, epoch, up, act_n, pas_n):", top[:20])
hist_s = np.zeros(65, int)
hist_r = np.zeros(65, int)
for lo in range(0, n, step):
    v = sim.nodes(lo, min(step, n - lo))
    hist_s += np.bincount(v["sent_n"], minlength=65)[:65]
    hist_r += np.bincount(v["recv_n"], minlength=65)[:65]
print("sent_n histogram (nonzero bins):", {i: int(c) for i, c in enumerate(hist_s) if c})
print("recv_n histogram (nonzero bins):", {i: int(c) for i, c in enumerate(hist_r) if c})
