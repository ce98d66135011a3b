"""HBM traffic record of the node-round kernels for one bench.py command,
from a FETCH_SIZE pass and a WRITE_SIZE pass of that same command
(profiles/run_pmc.sh).  Appends / replaces the record in
profiles/pmc_records.json, which bench.py reads back by its pmc_key.

Window: the `steps` timed rounds are the dispatches of each kernel before the
overlay-drain rounds bench.py runs after its window (overlay.rounds_drained).
Per round: the sum over the node-round kernels (k_relay, k_shuf, k_lite_half
or k_consume_lite, k_consume, k_ptq or k_ptl, k_pt; k_consume_pl for the
pluggable lines B and D, which drain no rounds after their window).

Units and corrections (profiles/calib/, measured on this MI355X): FETCH_SIZE
counts 64-B memory requests -- a random dword or a random 64-B record reads as
exactly 64 B, a fully coalesced 16-B-per-lane stream as half its bytes (128-B
requests tallied at 64 B, the guide's x2).  The node-round kernels read
random rows and records, so `traffic` = FETCH_SIZE + WRITE_SIZE (the
random-access calibration) and `traffic_upper` = 2 x FETCH_SIZE + WRITE_SIZE
(every read a 128-B request).
Usage: python profiles/pmc_record.py BENCH_JSON FETCH_CSV WRITE_CSV"""
import csv
import json
import os
import sys

KERNELS = ("k_relay(", "k_shuf(", "k_consume_lite(", "k_lite_half(", "k_term(", "k_consume(", "k_ptl(", "k_ptq(",
           "k_pt(", "k_consume_pl(")


def per_round(path, steps, tail, by=None):
    """bytes per timed round over the node-round kernels; `by` collects them
    per kernel"""
    rows = list(csv.DictReader(open(path)))
    tot = 0.0
    for k in KERNELS:
        kr = [r for r in rows if k in r["Kernel_Name"]]
        ids = sorted({int(r["Dispatch_Id"]) for r in kr})
        keep = set(ids[len(ids) - tail - steps:len(ids) - tail])
        b = sum(float(r["Counter_Value"]) for r in kr if int(r["Dispatch_Id"]) in keep) * 1024 / steps
        tot += b
        if by is not None and b:
            by[k.rstrip("(")] = by.get(k.rstrip("("), 0.0) + b
    return tot                         # (KiB counts -> bytes, per round)


def main():
    bench = json.load(open(sys.argv[1]))
    steps, tail = bench["steps"], bench.get("overlay", {}).get("rounds_drained", 0)
    by = {}
    fetch = per_round(sys.argv[2], steps, tail, by)
    write = per_round(sys.argv[3], steps, tail, by)
    rec = {"key": bench["pmc_key"],
           "traffic_per_launch": fetch + write,
           "traffic_upper_per_launch": 2 * fetch + write,
           "fetch_size_bytes": fetch, "write_size_bytes": write,
           "alg_bytes_per_launch": bench["roofline"]["alg_bytes_per_launch"],
           "per_kernel": by,              # FETCH_SIZE + WRITE_SIZE per round, by kernel
           # each kernel's algorithmic bytes per round (bench.py --kernel-counts:
           # its own nodes processed, deliveries, emissions) and counted / algorithmic
           "per_kernel_alg": bench.get("per_kernel_alg"),
           "per_kernel_excess": ({k: by[k] / a for k, a in bench["per_kernel_alg"].items() if a and k in by}
                                 if bench.get("per_kernel_alg") else None),
           "source": "FETCH_SIZE + WRITE_SIZE per timed round of the node-round kernels, separate "
                     "rocprofv3 --pmc passes of this command (profiles/run_pmc.sh); FETCH_SIZE uncorrected: "
                     "random 64-B requests count exactly (profiles/calib/)"}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pmc_records.json")
    try:
        recs = json.load(open(path))
    except (OSError, ValueError):
        recs = []
    recs = [r for r in recs if r.get("key") != rec["key"]] + [rec]
    json.dump(recs, open(path, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
