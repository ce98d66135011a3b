#!/bin/bash
# The other bench lines on the current source, with their PMC traffic
# records and kernel tables: E at 2^26 on SURVEY 8(d)'s schedule (the
# partition at phase rounds 150-169; a 140-round window from phase round 45
# covers the churn, the partition and the heal) and on round 3's (doubling:
# the partition inside the churn, 60 rounds), B, D, C at 2^24; SQ counters
# of E at 2^26; config C's overlay classified at 2^24 on the GPU.
# Usage (GPU box, repo root): bash profiles/r04/lines.sh TAG
TAG=${1:-lines}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
summ() {
python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]; o = d.get("overlay", {})
print(sys.argv[1].split("/")[-1], "%.3g" % d["value"], "ms/step %.3f phase %.3f frac %.4f step_frac %s traffic %s rel %s comps %s ovf %d" % (
    d["ms_per_step"], r["avg_launch_ms"], r["frac"], r.get("step_frac"), r.get("traffic"),
    o.get("tracked_broadcast_reliability"), o.get("components"), d["overflow"]))
PY
}
trace() {  # name, bench args...
  local n=$1; shift
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/tr_$n -o run --output-format csv -- \
    python3 -u $R/bench.py --no-cpu-baseline --no-check "$@" > $O/bench_$n.json 2> $O/$n.err || { echo "$n FAILED"; tail -5 $O/$n.err; exit 1; }
  cd $R
  cp $(find $O/tr_$n -name "*kernel_stats.csv" | head -1) $O/kernel_stats_$n.csv
  local T=$(find $O/tr_$n -name "*kernel_trace.csv" | head -1)
  local S=$(python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['steps'])" $O/bench_$n.json)
  local D=$(python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]).get('overlay',{}).get('rounds_drained',0))" $O/bench_$n.json)
  python3 profiles/round_kernels.py $T $S --tail $D > $O/kernels_$n.txt
  gzip -c $T > $O/kernel_trace_$n.csv.gz && rm -rf $O/tr_$n
  summ $O/bench_$n.json
  head -8 $O/kernels_$n.txt
}
E26S="--workload E --schedule survey --nodes 67108864 --steps 140 --warmup 5"
E26D="--workload E --schedule doubling --nodes 67108864 --steps 60 --warmup 5"
trace E26s $E26S || exit 1
trace E26d $E26D || exit 1
bash profiles/run_pmc.sh ${TAG}_E26s $E26S --no-check | tail -1 || exit 1
bash profiles/run_pmc.sh ${TAG}_B --workload B --steps 20 --warmup 5 | tail -1 || exit 1
bash profiles/run_pmc.sh ${TAG}_D --workload D --steps 20 --warmup 5 | tail -1 || exit 1
bash profiles/run_pmc.sh ${TAG}_C24 --nodes 16777216 --steps 20 --warmup 5 --no-check | tail -1 || exit 1
for n in B D; do timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $n --steps 20 --warmup 5 > $O/bench_$n.json 2> $O/$n.err && summ $O/bench_$n.json; done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-check --nodes 16777216 --steps 20 --warmup 5 > $O/bench_C24.json 2> $O/C24.err && summ $O/bench_C24.json
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-check $E26S > $O/bench_E26s_pmc.json 2> $O/E26s_pmc.err && summ $O/bench_E26s_pmc.json
bash profiles/sq_kernels.sh $TAG/sq_E26 --workload E --schedule survey --nodes 67108864 --steps 20 --warmup 5 > /dev/null && tail -7 $O/sq_E26/sq_kernels.txt
timeout -k 10 600 python3 -u tests/c_overlay.py --backend gpu --nodes 1048576 > $O/c_overlay_gpu.jsonl 2>&1
timeout -k 10 900 python3 -u tests/c_overlay.py --backend gpu --nodes 16777216 --points > $O/c_overlay_gpu24.jsonl 2>&1
tail -c 600 $O/c_overlay_gpu24.jsonl
