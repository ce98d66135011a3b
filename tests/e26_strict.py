"""Config E at its full size on one GPU as a property test (VERDICT r5 item
1b; BASELINE.json configs[4], the north star's 64M-node overlay): 2^26
nodes, HyParView + Plumtree on SURVEY 8(d)'s E schedule
(partisan_amd.workloads.BenchSchedule "E"/"survey" -- the doubling
bootstrap, 60 settle rounds, 0.2 N crashes over phase rounds 40-139, each
victim restarting and rejoining a live node the next round, a broadcast from
node 0 every 10 rounds, the half/half partition for phase rounds 150-169)
with cfg.strict = 1, so any fixed-table overflow fails the step
(PSIM_ECAPACITY).  The oracle cannot run at this size; the checks are
size-independent:
  * no overflow in any round (strict), every node up at the end;
  * messages conserved every round: what round r emits is delivered or
    dropped in round r + 1;
  * after the partition heals (phase round 180): a broadcast from node 0
    reaches >= 0.999 of the nodes within 40 rounds and never more than the
    largest component;
  * active links symmetric (>= 0.999 of them have their reverse).

Run directly (prints progress) or from tests/test_gpu_e26.py.  Exit 0 = ok."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

from partisan_amd import Simulator  # noqa: E402
from partisan_amd import workloads as W  # noqa: E402
from partisan_amd.sim import default_config  # noqa: E402

N = int(os.environ.get("PSIM_E26_NODES", 1 << 26))
SEED = 1
HEALED = 180                       # phase round: ten rounds after the partition ends
T0 = time.time()


def log(*a):
    print(f"[{time.time() - T0:7.1f}s]", *a, file=sys.stderr, flush=True)


def main():
    cfg = default_config(n_nodes=N, seed=SEED, device=0)
    cfg.strict = 1
    sim = Simulator(cfg)
    sched = W.BenchSchedule("E", "survey", N, SEED, 5)
    assert (sched.p_on, sched.p_off) == (150, 170)
    boot, until = sched.bootstrap()
    st = [sim.run_schedule(boot, until, extra=lambda r: r % 8 == 0 and log("bootstrap round", r))]
    log("bootstrap done at round", sim.round)
    i = 0
    while i < HEALED:
        sched.apply(sim, i)
        k = 1
        while i + k < HEALED and not sched.has_events(i + k):
            k += 1
        st.append(sim.step(k))
        i += k
        if i % 20 < k:
            log("phase round", i)
    # one more broadcast on the healed overlay, no further events
    assert sched.bcast_round(i)
    sched.apply(sim, i)
    st.append(sim.step(40))
    st = np.concatenate(st)
    h = sim.histograms()
    log("done,", len(st), "rounds")
    assert int(st["overflow"].sum()) == 0
    em = st["emitted"].sum(axis=1)
    got = st["delivered"].sum(axis=1) + st["dropped"]
    bad = np.flatnonzero(em[:-1] != got[1:])
    assert bad.size == 0, f"messages not conserved from round {int(st['round'][bad[0]])}"
    assert h["n_up"] == N, h["n_up"]
    rel = h["delivered"] / N
    assert rel >= 0.999 and h["delivered"] <= h["largest_component"], (rel, h["largest_component"])
    sym = h["symmetric_links"] / max(1, h["active_links"])
    assert sym >= 0.999, sym
    assert int(st["nodes_up"][-1]) == N
    print("E26 OK", {"nodes": N, "rounds": len(st), "strict": True, "overflow": 0, "reliability": round(rel, 6),
                     "symmetric": round(sym, 6), "components": int(h["components"]),
                     "msgs": int(st["emitted"].sum()), "exits": int(st["exits"].sum()),
                     "seconds": round(time.time() - T0, 1)}, flush=True)
    sim.close()


if __name__ == "__main__":
    main()
