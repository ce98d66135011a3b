"""Config E's survey schedule (tests/e26_strict.py's) with the bound-terms
diagnostic build (PSIM_LIB=bterms, PSIM_TRACE_BOUND=1): after every step the
library prints the outbox bound's terms summed over that step's rounds, and
this script prints the records the same rounds emitted beside them.
Usage (GPU box, repo root): PSIM_LIB=bterms PSIM_TRACE_BOUND=1 python
profiles/r06/bterms.py [log2 nodes]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from partisan_amd import Simulator  # noqa: E402
from partisan_amd import workloads as W  # noqa: E402
from partisan_amd.sim import default_config  # noqa: E402

N = 1 << int(sys.argv[1] if len(sys.argv) > 1 else 26)


def emitted(st):
    return int(st["emitted"].sum()), len(st), int(st["emitted"].sum(axis=1).max())


def main():
    cfg = default_config(n_nodes=N, seed=1, device=0)
    sim = Simulator(cfg)
    sched = W.BenchSchedule("E", "survey", N, 1, 5)
    boot, until = sched.bootstrap()
    st = sim.run_schedule(boot, until)
    print("bootstrap: emitted %d over %d rounds (max %d)" % emitted(st), file=sys.stderr, flush=True)
    i = 0
    while i < 200:
        sched.apply(sim, i)
        k = 1
        while i + k < 200 and i + k < 165 and not sched.has_events(i + k):
            k += 1
        st = sim.step(k)
        print("phase %d-%d: emitted %d over %d rounds (max %d)" % ((i, i + k - 1) + emitted(st)),
              file=sys.stderr, flush=True)
        i += k
    sim.close()


if __name__ == "__main__":
    main()
