#!/bin/bash
# The rank path's line (bench.py --rank-path: a one-rank RCCL communicator)
# under a kernel trace, with its batches traced (PSIM_TRACE_BATCH); then the
# local line for comparison.  Usage: bash profiles/r06/ranktrace.sh TAG
TAG=${1:-r6rt}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
PSIM_TRACE_BATCH=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rank-path --no-cpu-baseline > $O/bench_rank.json 2> $O/bench_rank.err || { tail -5 $O/bench_rank.err; exit 1; }
grep "batch of" $O/bench_rank.err | tail -12
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-check --steps 20 --warmup 5 --rank-path > $O/prof_rank.json 2> $O/prof_rank.err || { echo PROF FAILED; tail -5 $O/prof_rank.err; exit 1; }
cd $R
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
TAIL=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['overlay']['rounds_drained'])" $O/prof_rank.json)
python3 profiles/steady_kernels.py $T --steps 20 --tail $TAIL > $O/steady_rank.txt && head -30 $O/steady_rank.txt
gzip -c $T > $O/kernel_trace_rank.csv.gz && rm -rf $O/prof
python3 - $O <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/bench_rank.json")); r = d["roofline"]
print("rank %.4g node-rounds/s  ms/step %.4f  phase %.4f  x %s" % (d["value"], d["ms_per_step"], r["avg_launch_ms"], d.get("exchange")))
PY
