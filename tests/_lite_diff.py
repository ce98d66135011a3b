"""Debug tool (not a test): the GPU engine in lockstep with the oracle on a
scenario; at the first round whose stats differ, print the nodes whose
state differs, with the oracle's view of them before that round and their
inbox, and the GPU's after.  Usage: python tests/_lite_diff.py [scenario]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import _scenarios as S  # noqa: E402
from _oracle import Oracle  # noqa: E402
from partisan_amd import Simulator  # noqa: E402


class Lock:
    """drives both backends with the same calls; step() compares"""

    def __init__(self, cfg):
        self.g, self.o = Simulator(cfg), Oracle(cfg)
        self.cfg = cfg
        self.n = cfg.n_nodes

    def __getattr__(self, k):
        if k in ("join", "crash", "revive", "set_partition", "clear_partition", "broadcast", "set_bucket_table"):
            return lambda *a: (getattr(self.g, k)(*a), getattr(self.o, k)(*a))
        raise AttributeError(k)

    @property
    def round(self):
        return self.o.round

    grace = None

    def step(self, k=1):
        out = []
        for _ in range(k):
            before = self.o.nodes()
            inbox = self.o.inbox()
            go, oo = self.g.step(1), self.o.step(1)
            bad = [f for f in S.STAT_FIELDS if not np.array_equal(go[f], oo[f])]
            if bad and self.grace is None and bad == ["digest"]:
                print(f"round {int(oo['round'][0])}: only the digest differs; going on to a state difference")
                self.grace = 4
            if self.grace is not None:
                self.grace -= 1
                gn, on = self.g.nodes(), self.o.nodes()
                same = all(np.array_equal(gn[f], on[f]) for f in gn.dtype.names)
                if same and self.grace > 0:
                    out.append(oo)
                    continue
                bad = bad or ["(state)"]
            if bad:
                r = int(oo["round"][0])
                print(f"round {r}: stats differ in {bad}")
                for f in bad:
                    print("  gpu", go[f].tolist(), "\n  orc", oo[f].tolist())
                gn, on = self.g.nodes(), self.o.nodes()
                diff = np.nonzero([any(not np.array_equal(gn[f][i], on[f][i]) for f in gn.dtype.names)
                                   for i in range(self.n)])[0]
                print(f"  {len(diff)} nodes differ: {diff[:20].tolist()}")
                for i in diff[:4]:
                    b = before[i]
                    print(f"--- node {i}: before act {b['act'][:b['act_n']].tolist()} "
                          f"pas({b['pas_n']}) {b['pas'][:b['pas_n']].tolist()} rng {b['rng_ctr']}")
                    for m in inbox[inbox[:, 0] == i]:
                        print("    in", m.tolist())
                    for f in gn.dtype.names:
                        if not np.array_equal(gn[f][i], on[f][i]):
                            print(f"    {f}: gpu {np.asarray(gn[f][i]).tolist()}\n    {' ' * len(f)}  orc {np.asarray(on[f][i]).tolist()}")
                sys.exit(1)
            out.append(oo)
        return np.concatenate(out)

    run_schedule = Oracle.run_schedule


name = sys.argv[1] if len(sys.argv) > 1 else "e_miniature"
fn = getattr(S, name)
fn(Lock)
print("no difference")
