"""Per-round breakdown of the 1M-node workload: work counters and kernel
times, one line per round (diagnostic; run on the GPU box)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from partisan_amd import Simulator, workloads as W  # noqa: E402
from partisan_amd.sim import default_config  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 30
sim = Simulator(default_config(n_nodes=n, seed=1))
boot = W.doubling_join(n, 1)
sim.run_schedule(boot, boot[-1][0] + 61)
print("round proc deliv emit up | consume_ms prepare sort")
for i in range(rounds):
    if i % 10 == 0:
        sim.broadcast(0, i // 10)
    st = sim.step(1)[0]
    kt = sim.kernel_times()
    print(int(st["round"]), int(st["nodes_processed"]), int(st["delivered"].sum()),
          int(st["emitted"].sum()), int(st["nodes_up"]), "|",
          "%.3f %.3f %.3f" % (kt["consume"][0], kt["prepare"][0], kt["sort"][0]),
          "pt:", st["delivered"][9:14].tolist(), flush=True)
