"""Sum rocprofv3 --pmc counters per kernel from run_counter_collection.csv files.
Usage: python profiles/pmc_summary.py DIR [DIR...] [--kernel SUBSTR]"""
import csv
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    ksub = "k_consume"
    if "--kernel" in sys.argv:
        ksub = sys.argv[sys.argv.index("--kernel") + 1]
        args.remove(ksub)
    last = None                      # only the last K dispatches (the timed rounds)
    if "--last" in sys.argv:
        v = sys.argv[sys.argv.index("--last") + 1]
        last = int(v)
        args.remove(v)
    tot = defaultdict(float)
    disp = defaultdict(set)
    for d in args:
        with open(f"{d}/run_counter_collection.csv") as f:
            rows = [r for r in csv.DictReader(f) if ksub in r["Kernel_Name"]]
        if last:
            ids = sorted({int(r["Dispatch_Id"]) for r in rows})[-last:]
            keep = set(ids)
            rows = [r for r in rows if int(r["Dispatch_Id"]) in keep]
        for row in rows:
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[row["Counter_Name"]].add(row["Dispatch_Id"])
    for k in sorted(tot):
        n = len(disp[k])
        print(f"{k:24s} total {tot[k]:.4g}  per-dispatch {tot[k] / n:.4g}  ({n} dispatches)")
    if "SQ_WAVE_CYCLES" in tot:
        wc = tot["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"):
            if k in tot:
                print(f"{k} / SQ_WAVE_CYCLES = {tot[k] / wc:.3f}")


if __name__ == "__main__":
    main()
