"""Debug tool (not a test): k_lite_half against k_consume_lite
(PSIM_LITE_WAVE=1) in lockstep on one GPU; after every round the routed
records (the snapshot's inbox) are compared, and the first differing records
printed.  Usage: python tests/_lite_diff2.py [scenario]"""
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import _scenarios as S  # noqa: E402
from partisan_amd import Simulator  # noqa: E402

HEAD = 568          # SnapHead


def inbox(sim):
    b = sim.snapshot()
    m_in = struct.unpack_from("<I", b, HEAD + 8)[0]
    return np.frombuffer(b[len(b) - 64 * m_in:], np.uint32).reshape(-1, 16), m_in


class Lock:
    def __init__(self, cfg):
        import ctypes as C
        from partisan_amd import _abi
        c2 = _abi.PsimConfig.from_buffer_copy(cfg)
        os.environ["PSIM_LITE_WAVE"] = "1"
        self.old = Simulator(cfg)
        del os.environ["PSIM_LITE_WAVE"]
        self.new = Simulator(c2)
        self.n = cfg.n_nodes

    def __getattr__(self, k):
        if k in ("join", "crash", "revive", "set_partition", "clear_partition", "broadcast", "set_bucket_table"):
            return lambda *a: (getattr(self.old, k)(*a), getattr(self.new, k)(*a))
        raise AttributeError(k)

    @property
    def round(self):
        return self.old.round

    def step(self, k=1):
        out = []
        for _ in range(k):
            a, b = self.old.step(1), self.new.step(1)
            ia, na = inbox(self.old)
            ib, nb = inbox(self.new)
            r = int(a["round"][0])
            if na != nb or not np.array_equal(ia, ib):
                print(f"round {r}: routed records differ ({na} vs {nb})")
                ka = {tuple(x[:4].tolist()): x for x in ia}
                kb = {tuple(x[:4].tolist()): x for x in ib}
                shown = 0
                for key in sorted(set(ka) | set(kb)):
                    x, y = ka.get(key), kb.get(key)
                    if x is None or y is None or not np.array_equal(x, y):
                        print("  old", None if x is None else x.tolist())
                        print("  new", None if y is None else y.tolist())
                        shown += 1
                        if shown >= 12:
                            break
                if shown == 0:
                    print("  same records, different order")
                    d = np.nonzero((ia != ib).any(1))[0]
                    for i in d[:6]:
                        print("  at", i, "old", ia[i].tolist(), "\n        new", ib[i].tolist())
                sys.exit(1)
            out.append(a)
        return np.concatenate(out)

    def run_schedule(self, schedule, until_round, extra=None):
        ev = {}
        for r, ids, contacts in schedule:
            ev.setdefault(r, []).append((ids, contacts))
        st = []
        while self.round < until_round:
            r = self.round
            for ids, contacts in ev.get(r, []):
                self.join(ids, contacts)
            if extra is not None:
                extra(r)
            st.append(self.step(1))
        return np.concatenate(st)


name = sys.argv[1] if len(sys.argv) > 1 else "e_miniature"
getattr(S, name)(Lock)
print("no difference")
