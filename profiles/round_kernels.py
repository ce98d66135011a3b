"""Per-round kernel time by kernel over the last STEPS rounds of a kernel
trace (a round starts at its k_node_prep; the event kernels launched before
it count to the round before): mean us per round per kernel name, sorted.
Usage: python profiles/round_kernels.py run_kernel_trace.csv [STEPS] [--tail TAIL]
(TAIL: rounds after the window to skip, e.g. bench.py's overlay drain,
overlay.rounds_drained)"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else 60
tail = int(sys.argv[sys.argv.index("--tail") + 1]) if "--tail" in sys.argv else 0
rounds, cur = [], None
for r in rows:
    name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "").strip()
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "k_node_prep" in name:
        cur = {"_start": int(r["Start_Timestamp"])}
        rounds.append(cur)
    if cur is not None:
        cur[name] = cur.get(name, 0.0) + d
        cur["_end"] = int(r["End_Timestamp"])
rounds = rounds[:-1]                  # (the last segment may hold the teardown's kernels)
if tail:
    rounds = rounds[:-tail]
last = rounds[-steps:]
tot = {}
for c in last:
    for k, v in c.items():
        if not k.startswith("_"):
            tot[k] = tot.get(k, 0.0) + v / len(last)
span = sum((c["_end"] - c["_start"]) / 1e3 for c in last) / len(last)
busy = sum(tot.values())
print(f"{len(last)} rounds: kernel time {busy / 1e3:.2f} ms/round, first-to-last kernel span {span / 1e3:.2f} ms/round")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {v / 1e3:9.3f} ms  {v / busy * 100:5.1f} %  {k}")
