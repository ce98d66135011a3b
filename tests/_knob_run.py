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

gs, gst = S.e_miniature(Simulator)
os_, ost = S.e_miniature(Oracle)
S.compare_stats(gst, ost)
S.compare_nodes(gs.nodes(), os_.nodes())
print("knobs", {k: v for k, v in os.environ.items() if k.startswith("PSIM_")}, "identical over", len(gst), "rounds")
