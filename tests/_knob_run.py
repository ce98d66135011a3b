"""Child process of tests/test_gpu_knobs.py: config E in miniature (churn,
restarts, a partition, broadcasts) on the GPU under whatever PSIM_* launch /
route / scan knobs the environment sets, against the oracle.  Exit 0 = every
round's stats and the final node state identical."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import _scenarios as S  # noqa: E402
from _oracle import Oracle  # noqa: E402
from partisan_amd import Simulator  # noqa: E402

# PSIM_KNOB_PATH: the engine path the scenario runs through -- "local" (one
# shard), "loopbackN" (N loopback ranks: the rank path), "rccl1" (a one-rank
# RCCL communicator)
path = os.environ.get("PSIM_KNOB_PATH", "local")
if path.startswith("loopback"):
    from _loopback import LoopbackRanks
    make = lambda cfg: LoopbackRanks(cfg, int(path[len("loopback"):]))  # noqa: E731
elif path == "rccl1":
    from partisan_amd.sim import comm_id

    def make(cfg):
        c = type(cfg).from_buffer_copy(cfg)
        c.shard_world, c.shard_rank, c.n_shards = 1, 0, 1
        return Simulator(c, comm=comm_id())
else:
    make = Simulator
gs, gst = S.e_miniature(make)
os_, ost = S.e_miniature(Oracle)
S.compare_stats(gst, ost)
S.compare_nodes(gs.nodes(), os_.nodes())
print("knobs", {k: v for k, v in os.environ.items() if k.startswith("PSIM_")}, "identical over", len(gst), "rounds")
