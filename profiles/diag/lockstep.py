"""Diagnostic: any scenario of tests/_scenarios.py on the GPU and the oracle
in lock step -- every step() is run one round at a time on both, stats and
node views compared after each round; the first differing round prints the
differing stats fields, nodes and fields (the first few), then exits 1.
Usage: python profiles/diag/lockstep.py SCENARIO [SCENARIO ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import _scenarios as S  # noqa: E402
from _oracle import Oracle  # noqa: E402
from partisan_amd import Simulator  # noqa: E402
from partisan_amd.sim import _Driver  # noqa: E402

STATS = ("emitted", "delivered", "exits", "send_fail", "digest", "first_deliveries", "nodes_processed")


class Diverged(Exception):
    pass


def show(v, i, f):
    x = v[f][i]
    return x.tolist() if hasattr(x, "tolist") else x


class Lockstep:
    def __init__(self, cfg):
        self.g, self.o = Simulator(cfg), Oracle(cfg)
        self.n = self.g.n

    def __getattr__(self, name):
        fg, fo = getattr(self.g, name), getattr(self.o, name)
        if not callable(fg):
            return fg

        def both(*a, **kw):
            r = fg(*a, **kw)
            fo(*a, **kw)
            return r
        return both

    run_schedule = _Driver.run_schedule          # (through step below: lock step)

    def step(self, k=1):
        out = []
        for _ in range(k):
            prev, ib = self.o.nodes(), self.o.inbox()
            sg, so = self.g.step(1), self.o.step(1)
            out.append(sg)
            r = int(sg["round"][0])
            ds = [f for f in STATS if not np.array_equal(sg[f], so[f])]
            g, o = self.g.nodes(), self.o.nodes()
            bad = [(f, np.nonzero((g[f] != o[f]).reshape(self.n, -1).any(1))[0]) for f in g.dtype.names]
            bad = [(f, d) for f, d in bad if len(d)]
            if ds or bad:
                print(f"round {r}: stats differ in {ds}; node fields: {[(f, len(d)) for f, d in bad]}")
                for f in ds:
                    print(f"  {f}: gpu {sg[f].tolist()} oracle {so[f].tolist()}")
                ids = sorted(set(int(x) for _, d in bad for x in d[:4]))[:6]
                for i in ids:
                    for f, _ in bad:
                        if not np.array_equal(g[f][i], o[f][i]):
                            print(f"  node {i} {f}: gpu {show(g, i, f)} oracle {show(o, i, f)}")
                for i in ids:
                    p = prev[i]
                    print(f"  node {i} before: up {p['up']} start {p['start_round']} act {p['act'][:p['act_n']].tolist()} "
                          f"pas {p['pas'][:p['pas_n']].tolist()} conn {[hex(c) for c in p['conn'][:p['conn_n']]]}")
                    peers = set(int(x) for x in p['act'][:p['act_n']]) | set(int(c) & 0x7FFFFFFF for c in p['conn'][:p['conn_n']])
                    print(f"    peers up before/after: {[(q, int(prev['up'][q]), int(o['up'][q])) for q in sorted(peers) if q < self.n]}")
                    for m in ib[ib[:, 0] == i]:
                        print(f"    in: src {m[1]} seq {m[2]} type {m[3] & 0xFF} ttl {(m[3] >> 8) & 0xFF} "
                              f"a0 {m[4]} a1 {m[5]} a2 {m[6]} a3 {m[7]} ex {m[8:8 + ((m[3] >> 16) & 0xFF)].tolist()}")
                raise Diverged(r)
        return np.concatenate(out)


if __name__ == "__main__":
    rc = 0
    for name in sys.argv[1:]:
        try:
            getattr(S, name)(Lockstep)
            print(f"{name}: identical")
        except Diverged:
            rc = 1
    sys.exit(rc)
