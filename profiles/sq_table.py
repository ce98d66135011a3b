"""Per-kernel SQ counter table over the timed rounds of one bench.py run
(profiles/sq_kernels.sh).  Usage: python profiles/sq_table.py counter_collection.csv bench.json
The timed rounds are each kernel's dispatches before the overlay drain's
(bench.json overlay.rounds_drained) and after the warmup; per dispatch values
are averaged over those rounds."""
import csv
import json
import sys
from collections import defaultdict

KERNELS = ["k_relay", "k_shuf", "k_consume_lite", "k_lite_half", "k_term", "k_consume", "k_ptl", "k_ptq", "k_pt",
           "k_consume_pl"]


def kname(s):
    s = s.replace("(anonymous namespace)::", "")
    s = s.split("(")[0].split("::")[-1]
    return s


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    steps, tail = b["steps"], b.get("overlay", {}).get("rounds_drained", 0)
    per = defaultdict(lambda: defaultdict(dict))       # kernel -> dispatch -> counter -> value
    for r in rows:
        k = kname(r["Kernel_Name"])
        if k in KERNELS:
            d = per[k][int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print(f"# {b['config'].get('schedule', '?')} schedule, {b['config']['nodes']} nodes, {steps} timed rounds "
          f"(before the last {tail} dispatches); per-round averages")
    print(f"{'kernel':16s} {'waves':>9s} {'VALU/wave':>9s} {'SALU/wave':>9s} {'LDS/wave':>8s} "
          f"{'wait%':>6s} {'issue%':>6s} {'waves/SIMD':>10s} {'Mcycles':>8s}")
    for k in KERNELS:
        ds = sorted(per[k])
        keep = ds[len(ds) - tail - steps:len(ds) - tail] if len(ds) > tail + steps else ds
        if not keep:
            continue
        t = defaultdict(float)
        for i in keep:
            for c, v in per[k][i].items():
                t[c] += v / len(keep)
        w = max(1.0, t["SQ_WAVES"])
        wc = max(1.0, t["SQ_WAVE_CYCLES"])
        cyc = t["GRBM_GUI_ACTIVE"] / 8
        occ = 4 * wc / (cyc * 1024) if cyc else 0.0
        print(f"{k:16s} {w:9.0f} {t['SQ_INSTS_VALU'] / w:9.0f} {t['SQ_INSTS_SALU'] / w:9.0f} "
              f"{t['SQ_INSTS_LDS'] / w:8.0f} {100 * t['SQ_WAIT_ANY'] / wc:6.1f} "
              f"{100 * t['SQ_ACTIVE_INST_ANY'] / wc:6.1f} {occ:10.2f} {cyc / 1e6:8.3f}")


if __name__ == "__main__":
    main()
