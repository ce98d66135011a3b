"""Diagnostic: the churn_partition scenario on the GPU and the oracle side
by side, node views compared after every round from --from on; prints the
first differing nodes and fields (then stops).
Usage: python profiles/diag/q11_diff.py [--n 2048] [--from 40] [--to 60]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from _oracle import Oracle  # noqa: E402
from partisan_amd import Simulator, workloads as W  # noqa: E402
from partisan_amd.sim import default_config  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=2048)
p.add_argument("--seed", type=int, default=5)
p.add_argument("--from", dest="first", type=int, default=40)
p.add_argument("--to", type=int, default=60)
a = p.parse_args()
n, seed = a.n, a.seed
sims = [Simulator(default_config(n_nodes=n, seed=seed)), Oracle(default_config(n_nodes=n, seed=seed))]
churn = {r: (v, c) for r, v, c in W.churn_schedule(n, seed, 0.2, 40, 40)}
part = W.half_partition(n)
joins = {r: (i, c) for r, i, c in W.doubling_join(n, seed)}
k = 0
for r in range(a.to):
    for s in sims:
        if r in joins:
            s.join(*joins[r])
        if r in churn:
            s.crash(churn[r][0])
            s.join(churn[r][0], churn[r][1])
        if r == 90:
            s.set_partition(part)
        if r == 100:
            s.clear_partition()
        if r >= 30 and (r - 30) % 10 == 0:
            s.broadcast(0, k % 0x10000)
    if r >= 30 and (r - 30) % 10 == 0:
        k += 1
    st = [s.step(1)[0] for s in sims]
    diff_st = [f for f in ("emitted", "delivered", "exits", "send_fail", "digest") if not np.array_equal(st[0][f], st[1][f])]
    if r < a.first and not diff_st:
        continue
    g, o = sims[0].nodes(), sims[1].nodes()
    bad = []
    for f in g.dtype.names:
        d = np.nonzero((g[f] != o[f]).reshape(n, -1).any(1))[0]
        if len(d):
            bad.append((f, d))
    print(f"round {r}: stats differ in {diff_st}; node fields differing: {[(f, len(d)) for f, d in bad]}", flush=True)
    if bad:
        ids = sorted(set(int(x) for _, d in bad for x in d[:5]))[:6]
        for i in ids:
            for f, _ in bad:
                if not np.array_equal(g[f][i], o[f][i]):
                    print(f"  node {i} {f}: gpu {g[f][i].tolist() if hasattr(g[f][i], 'tolist') else g[f][i]} "
                          f"| oracle {o[f][i].tolist() if hasattr(o[f][i], 'tolist') else o[f][i]}")
            for f in ("act_n", "act", "conn_n", "conn", "pas_n", "start_round", "up"):
                print(f"    {f}: gpu {g[f][i].tolist() if hasattr(g[f][i], 'tolist') else g[f][i]} | oracle {o[f][i].tolist() if hasattr(o[f][i], 'tolist') else o[f][i]}")
        break
    if diff_st:
        break
