"""Config D's HyParView half: HyParView + Plumtree on C's survey schedule at
2^24 nodes over 8 loopback ranks against the one-shard engine, with C's
overlay properties (tests/c24_loopback.py, a child process whose progress
goes to gpurun_out/c24_progress.log)."""
import gc
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_c24_eight_loopback_ranks_equal_one_shard():
    gc.collect()                                  # (handles of earlier tests released)
    out = os.path.join(os.path.dirname(HERE), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "c24_progress.log"), "w") as err:
        r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "c24_loopback.py")], stdout=subprocess.PIPE,
                           stderr=err, text=True, timeout=1000)
    assert r.returncode == 0 and "C24 OK" in r.stdout, r.stdout[-2000:]
