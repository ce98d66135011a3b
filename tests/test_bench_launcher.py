"""bench.py's multi-GPU launcher on CPU (gloo, --dry-run): `--gpus N`
without a launcher starts N ranks itself, they rendezvous, time the same
barrier-bracketed window and rank 0 prints one line with n_gpus = N; a
failing rank fails the run instead of hanging it; a WORLD_SIZE that
disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True,
                          timeout=timeout)


def test_launcher_starts_n_ranks():
    r = _run(["--gpus", "3", "--dry-run", "--steps", "7", "--warmup", "2"])
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout                 # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 3 and out["ranks"] == 3 and out["steps"] == 7 and out["warmup"] == 2


def test_launcher_failing_rank_fails_run():
    r = _run(["--gpus", "2", "--dry-run"], env={"PSIM_BENCH_FAIL_RANK": "1"})
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--dry-run"], env={"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_single_rank_dry_run():
    r = _run(["--dry-run", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1
