"""Diagnostic: first round where G virtual shards and one shard differ
(per-round stats incl. the record digest) for a doubling bootstrap of N
nodes.  Usage: python profiles/diag/shard_diverge.py N G [rounds]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import _scenarios as S  # noqa: E402
from partisan_amd import Simulator  # noqa: E402

n, g = int(sys.argv[1]), int(sys.argv[2])
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 40


def make(shards):
    def f(cfg):
        cfg.n_shards = shards
        cfg.device = 0
        return Simulator(cfg)
    return f


a, ast = S.doubling(make(1), n, 7, rounds)
b, bst = S.doubling(make(g), n, 7, rounds)
first = None
for f in S.STAT_FIELDS:
    d = np.nonzero((ast[f] != bst[f]).reshape(len(ast), -1).any(1))[0]
    if d.size:
        r = int(d[0])
        print(f"{f}: first differs at round {r}: one={ast[f][r]} sharded={bst[f][r]}")
        first = r if first is None else min(first, r)
print(f"N={n} G={g} rounds={rounds}: first differing round {first}")
for r in range(max(0, (first or 0) - 2), min(rounds, (first or 0) + 2)):
    print(r, "emitted", ast["emitted"][r][:9].tolist(), bst["emitted"][r][:9].tolist(),
          "proc", int(ast["nodes_processed"][r]), int(bst["nodes_processed"][r]),
          "ovf", int(ast["overflow"][r]), int(bst["overflow"][r]))
