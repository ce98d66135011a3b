"""The engine's measurement knobs change launch shapes and algorithms, never
results: another route bucket width (PSIM_ROUTE_WSHIFT), the route's
large-bucket path for every bucket (PSIM_ROUTE_REG=0), other grids for
every node-round kernel (PSIM_*_GRID), the HyParView kernels one after
another or side by side (PSIM_CONCURRENT_PHASE), the four-pass route instead
of the fused one (PSIM_ROUTE_FUSED=0), the wave-per-node
lite kernel instead of the two-nodes-per-wave one (PSIM_LITE_WAVE), the rank
path's exact rounds instead of its batches (PSIM_NO_RANK_BATCH) must
reproduce the oracle bit for bit.  The knobs are read once per process, so each set runs in
a child process (tests/_knob_run.py)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("knobs", [
    {"PSIM_ROUTE_WSHIFT": "12"},
    {"PSIM_ROUTE_REG": "0", "PSIM_ROUTE_BLOCKS": "7"},
    {"PSIM_LITE_WAVE": "1"},
    {"PSIM_LITE_GRID": "x1", "PSIM_PTL_GRID": "x2", "PSIM_PT_GRID": "x2", "PSIM_CONSUME_GRID": "x2"},
    {"PSIM_CONCURRENT_PHASE": "1"},
    {"PSIM_PTL_GRID": "x1"},
    {"PSIM_ROUTE_FUSED": "0"},
    # the rank path's exact rounds (no batches: the counts read back on the
    # host every round) against its batches of fixed-size messages
    {"PSIM_NO_RANK_BATCH": "1", "PSIM_KNOB_PATH": "loopback3"},
    {"PSIM_NO_RANK_BATCH": "1", "PSIM_KNOB_PATH": "rccl1"},
    {"PSIM_KNOB_PATH": "rccl1"},
])
def test_knobs_keep_parity(knobs):
    env = dict(os.environ, **knobs)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "_knob_run.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "identical" in r.stdout
