"""Average duration of a kernel over the bench's timed dispatches, from a
rocprofv3 kernel trace: the last STEPS dispatches of the kernel are the timed
rounds of bench.py once the TAIL overlay-drain dispatches after them are
skipped (warmup and bootstrap rounds come first; bench.py OVERLAY_DRAIN = 40).
Usage: python profiles/timed_avg.py run_kernel_trace.csv [--kernel k_consume] [--steps 50] [--tail 40]"""
import csv
import sys


def main():
    path = sys.argv[1]
    kern = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "k_consume("
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 50
    tail = int(sys.argv[sys.argv.index("--tail") + 1]) if "--tail" in sys.argv else 40
    rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows[len(rows) - tail - steps:len(rows) - tail]]
    print(f"{kern}: {len(rows)} dispatches; last {len(d)} (timed rounds) average {sum(d) / len(d):.4f} ms, "
          f"min {min(d):.4f}, max {max(d):.4f}")


if __name__ == "__main__":
    main()
