"""Per-round device time of every kernel over the bench's timed rounds, from a
rocprofv3 kernel trace: the window opens at the STEPS-th last k_consume
dispatch (the timed rounds come last) and each kernel's summed duration is
divided by STEPS.  Also the window's wall span per round (gaps included).
Rounds after the window (bench's overlay drain, `--tail`, from the bench
line's overlay.rounds_drained) are excluded.
Usage: python profiles/steady_kernels.py run_kernel_trace.csv [--steps 50] [--tail 40]"""
import collections
import csv
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    if "rocprim" in name:
        for tag in ("onesweep", "block_sort", "merge_sort", "lookback", "scan", "partition", "histogram",
                    "radix_sort"):
            if tag in name:
                return "rocprim:" + tag
        return "rocprim"
    return name


def main():
    path = sys.argv[1]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 50
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tail = int(sys.argv[sys.argv.index("--tail") + 1]) if "--tail" in sys.argv else 0
    cons = [i for i, r in enumerate(rows) if "k_consume(" in r["Kernel_Name"]]
    if tail:
        cons = cons[:-tail]
    first = cons[-steps]
    # the window: from the end of the round before the first timed consume
    # to the end of the last timed one
    prev = cons[-steps - 1] if len(cons) > steps else 0
    win = rows[prev + 1:cons[-1] + 1]
    tot = collections.Counter()
    calls = collections.Counter()
    for r in win:
        k = short(r["Kernel_Name"])
        tot[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        calls[k] += 1
    span = int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])
    busy = sum(tot.values())
    print(f"timed rounds {steps}: wall {span / steps / 1e6:.4f} ms/round, kernels {busy / steps / 1e6:.4f} ms/round")
    for k, t in tot.most_common():
        print(f"  {k:40s} {calls[k] / steps:5.1f}/round {t / steps / 1e3:9.1f} us/round")
    if "--per-round" in sys.argv:                 # the node-round kernels of each timed round
        print("per round (us): k_relay k_consume k_pt")
        cur = {}
        for r in win:
            k = short(r["Kernel_Name"]).replace("psim::", "")
            if k in ("k_relay", "k_consume", "k_pt"):
                cur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                if k == "k_pt" or (k == "k_consume" and "k_pt" not in cur and False):
                    print(f"  {cur.get('k_relay', 0):7.1f} {cur.get('k_consume', 0):7.1f} {cur.get('k_pt', 0):7.1f}")
                    cur = {}
    _ = first


if __name__ == "__main__":
    main()
