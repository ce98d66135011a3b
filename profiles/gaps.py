"""Idle gaps between consecutive kernels over the timed rounds of a rocprofv3
kernel trace (csv or csv.gz), summed per (previous, next) kernel pair.
Usage: python profiles/gaps.py run_kernel_trace.csv[.gz] [--steps 20]"""
import collections
import csv
import gzip
import sys


def nm(r):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if "rocprim" in n:
        for t in ("onesweep", "lookback", "scan", "partition", "merge"):
            if t in n:
                return "rocprim:" + t
    return n[-30:]


def main():
    path = sys.argv[1]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 20
    op = gzip.open if path.endswith(".gz") else open
    rows = list(csv.DictReader(op(path, "rt")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cons = [i for i, r in enumerate(rows) if "k_consume(" in r["Kernel_Name"]]
    win = rows[cons[-steps - 1] + 1:cons[-1] + 1]
    gaps, cnt = collections.Counter(), collections.Counter()
    for a, b in zip(win, win[1:]):
        k = (nm(a), nm(b))
        gaps[k] += int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
        cnt[k] += 1
    print("idle per round us %.1f" % (sum(gaps.values()) / steps / 1e3))
    for k, g in gaps.most_common(12):
        print(f"{g / steps / 1e3:8.1f} us/round  x{cnt[k] / steps:.1f}  {k[0]} -> {k[1]}")


if __name__ == "__main__":
    main()
