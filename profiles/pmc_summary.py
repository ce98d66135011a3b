"""Sum rocprofv3 --pmc counters of the node-round kernels per timed round,
from run_counter_collection.csv files.
Usage: python profiles/pmc_summary.py DIR [DIR...] [--kernels k_relay(,k_consume(]
                                       [--rounds 10] [--tail 40]
The timed rounds are the ROUNDS dispatches of each kernel before the TAIL
overlay-drain dispatches at the end of bench.py (OVERLAY_DRAIN = 40)."""
import csv
import sys
from collections import defaultdict


def opt(name, default):
    if name in sys.argv:
        v = sys.argv[sys.argv.index(name) + 1]
        return v
    return default


def main():
    flags = {"--kernels", "--rounds", "--tail"}
    args, skip = [], False
    for a in sys.argv[1:]:
        if skip:
            skip = False
            continue
        if a in flags:
            skip = True
            continue
        args.append(a)
    kernels = opt("--kernels", "k_relay(,k_consume(").split(",")
    rounds = int(opt("--rounds", "10"))
    tail = int(opt("--tail", "40"))
    tot = defaultdict(float)
    for d in args:
        with open(f"{d}/run_counter_collection.csv") as f:
            rows = list(csv.DictReader(f))
        for k in kernels:
            kr = [r for r in rows if k in r["Kernel_Name"]]
            ids = sorted({int(r["Dispatch_Id"]) for r in kr})
            keep = set(ids[len(ids) - tail - rounds:len(ids) - tail])
            for r in kr:
                if int(r["Dispatch_Id"]) in keep:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f"# kernels {','.join(kernels)}; {rounds} timed rounds before the last {tail} dispatches")
    for k in sorted(tot):
        print(f"{k:24s} total {tot[k]:.4g}  per-round {tot[k] / rounds:.4g}  ({rounds} rounds)")
    if "SQ_WAVE_CYCLES" in tot:
        wc = tot["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"):
            if k in tot:
                print(f"{k} / SQ_WAVE_CYCLES = {tot[k] / wc:.3f}")


if __name__ == "__main__":
    main()
