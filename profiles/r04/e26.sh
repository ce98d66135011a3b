#!/bin/bash
# Config E at 2^26 nodes: the kernel trace of round 3's line (doubling
# schedule, 60 rounds), SQ counters over a 20-round window, and the SURVEY
# 8(d) E line (partition at phase rounds 150-169, after the churn) whose
# 140-round window reaches past the heal.
# Usage (GPU box, repo root): bash profiles/r04/e26.sh TAG [skip-survey]
TAG=${1:-e26}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- \
  python3 -u $R/bench.py --workload E --schedule doubling --nodes 67108864 --steps 60 --warmup 5 --no-cpu-baseline --no-check \
  > $O/bench_E26.json 2> $O/E26.err || { echo "TRACE FAILED"; tail -5 $O/E26.err; exit 1; }
T=$(find $O/tr -name "*kernel_trace.csv" | head -1)
S=$(find $O/tr -name "*kernel_stats.csv" | head -1)
cp $S $O/kernel_stats.csv
python3 $R/profiles/round_kernels.py $T 60 --tail 40 > $O/e26_kernels.txt && head -16 $O/e26_kernels.txt
gzip -c $T > $O/kernel_trace.csv.gz && rm -rf $O/tr
cd $R
bash profiles/sq_kernels.sh $TAG/sq --workload E --schedule doubling --nodes 67108864 --steps 20 --warmup 5 > /dev/null || exit 1
tail -7 gpurun_out/$TAG/sq/sq_kernels.txt
[ "$2" = "skip-survey" ] && exit 0
timeout -k 10 420 python3 -u bench.py --workload E --schedule survey --nodes 67108864 --steps 140 --warmup 5 --no-cpu-baseline --no-check \
  > $O/bench_E26s.json 2> $O/E26s.err || { echo "SURVEY E FAILED"; tail -5 $O/E26s.err; exit 1; }
for f in bench_E26 bench_E26s; do
python3 - $O/$f.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]; o = d["overlay"]
print(sys.argv[1].split("/")[-1], "%.3g" % d["value"], "ms/step %.2f phase %.2f frac %.4f step_frac %.4f rel %.5f comps %d ovf %d"
      % (d["ms_per_step"], r["avg_launch_ms"], r["frac"], r["step_frac"], o["tracked_broadcast_reliability"], o["components"], d["overflow"]))
PY
done
