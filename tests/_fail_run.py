"""Child process of tests/test_gpu_parity.py::test_failed_step_poisons_until_restore:
PSIM_TEST_FAIL_ROUND (read once per process) makes round 50 fail half-way
with PSIM_ENOMEM, after its events reached the device.  The handle then
answers PSIM_ESTATE to every psim_step (include/partisan_gpu_sim.h) until a
snapshot is restored into it; after the restore it runs, identically to a
handle that never failed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import _scenarios as S  # noqa: E402
from partisan_amd import Simulator  # noqa: E402
from partisan_amd.sim import SimError, default_config  # noqa: E402

assert os.environ.get("PSIM_TEST_FAIL_ROUND") == "50"
sim, _ = S.doubling(Simulator, 2048, 4, 40)
snap = sim.snapshot()
sim.step(10)                                   # rounds 40-49
sim.broadcast(0, 3)
try:
    sim.step(5)                                # round 50 fails
    raise SystemExit("round 50 did not fail")
except SimError as e:
    assert "allocation" in str(e) or "memory" in str(e), e
for _ in range(2):
    try:
        sim.step(1)
        raise SystemExit("a failed handle stepped again")
    except SimError as e:
        assert "state" in str(e), e
sim.restore(snap)                              # round 40 again: back in service
assert sim.round == 40
a = sim.step(9)                                # rounds 40-48 (round 50 would fail again)
ref = Simulator(default_config(n_nodes=2048, seed=4))
ref.restore(snap)
b = ref.step(9)
S.compare_stats(a, b)
S.compare_nodes(sim.nodes(), ref.nodes())
# a snapshot is refused by a handle with another view-order table
other = Simulator(default_config(n_nodes=2048, seed=4))
other.set_bucket_table(S.random_buckets(2048, 5))
try:
    other.restore(snap)
    raise SystemExit("a snapshot restored under another table")
except SimError as e:
    assert "invalid" in str(e), e
print("failed step: ESTATE until restore; restore under another table refused")
