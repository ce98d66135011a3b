"""The measurement tooling around bench.py (CPU only): the CPU-share record
of the baseline and the PMC traffic record's per-round, per-kernel sums
(profiles/pmc_record.py) over a synthetic counter file."""
import csv
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def test_cpu_share_records_quota_affinity_and_env():
    import bench
    c = bench.cpu_share()
    assert c["affinity_cpus"] == len(os.sched_getaffinity(0))
    assert c["nproc"] == os.cpu_count()
    assert "cgroup_cpu_max" in c and "env" in c
    q = c["cgroup_cpu_max"]
    if q is not None:
        assert q["value"] and (q["quota_cpus"] is None or q["quota_cpus"] > 0)


def _counters(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_pmc_record_sums_the_timed_rounds_per_kernel(tmp_path):
    # 3 rounds of two kernels, then 1 drain round; steps = 2: the record is
    # the mean of rounds 2 and 3, per kernel and in total (KiB -> bytes)
    rows, did = [], 0
    for rnd, (a, b) in enumerate([(100, 10), (200, 20), (300, 40), (999, 999)]):
        for k, v in (("psim::k_relay(psim::RoundArgs)", a), ("psim::k_ptl(psim::RoundArgs)", b)):
            did += 1
            rows.append({"Dispatch_Id": did, "Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": v})
    fetch, write = tmp_path / "f.csv", tmp_path / "w.csv"
    _counters(fetch, rows)
    _counters(write, [dict(r, Counter_Name="WRITE_SIZE", Counter_Value=1) for r in rows])
    bench_json = tmp_path / "b.json"
    bench_json.write_text(json.dumps({"steps": 2, "overlay": {"rounds_drained": 1},
                                      "pmc_key": {"test": True}, "roofline": {"alg_bytes_per_launch": 1.0}}))
    env = dict(os.environ)
    records = os.path.join(ROOT, "profiles", "pmc_records.json")
    before = open(records).read()
    try:
        out = subprocess.run([sys.executable, os.path.join(ROOT, "profiles", "pmc_record.py"), str(bench_json),
                              str(fetch), str(write)], capture_output=True, text=True, env=env, check=True).stdout
    finally:
        with open(records, "w") as f:                 # (the committed records stay as they were)
            f.write(before)
    rec = json.loads(out)
    assert rec["fetch_size_bytes"] == (200 + 300 + 20 + 40) / 2 * 1024
    assert rec["write_size_bytes"] == 4 / 2 * 1024
    assert rec["per_kernel"]["k_relay"] == ((200 + 300) / 2 + 1) * 1024
    assert rec["per_kernel"]["k_ptl"] == ((20 + 40) / 2 + 1) * 1024
    assert rec["traffic_per_launch"] == rec["fetch_size_bytes"] + rec["write_size_bytes"]
