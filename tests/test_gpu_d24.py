"""Config D (SCAMP v2, c = 5) at its full 2^24 nodes over 8 loopback ranks
against the one-shard engine (tests/d24_loopback.py, a child process whose
progress goes to gpurun_out/d24_progress.log)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_d24_eight_loopback_ranks_equal_one_shard():
    out = os.path.join(os.path.dirname(HERE), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "d24_progress.log"), "w") as err:
        r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "d24_loopback.py")], stdout=subprocess.PIPE,
                           stderr=err, text=True, timeout=900)
    assert r.returncode == 0 and "D24 OK" in r.stdout, r.stdout[-2000:]
