"""Config E at its full 2^26 nodes on one GPU with cfg.strict = 1, as
size-independent properties (tests/e26_strict.py, a child process whose
progress goes to gpurun_out/e26_progress.log): no overflow, conservation
every round, reliability >= 0.999 after the partition heals, symmetric
active links."""
import gc
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_e26_survey_schedule_strict_properties():
    gc.collect()                                  # (handles of earlier tests released)
    out = os.path.join(os.path.dirname(HERE), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "e26_progress.log"), "w") as err:
        r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "e26_strict.py")], stdout=subprocess.PIPE,
                           stderr=err, text=True, timeout=1000)
    assert r.returncode == 0 and "E26 OK" in r.stdout, r.stdout[-2000:]
