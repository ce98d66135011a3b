#!/bin/bash
# Kernel-trace of a short bench run and the per-round kernel breakdown of its
# timed rounds (the trace itself is deleted; the summary is kept).
# Usage (on the box, repo root): [STEPS=20] bash profiles/prof_steady.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 "$@" > $O/bench.json 2> $O/prof.err || { echo PROF FAILED; tail -20 $O/prof.err; exit 1; }
cd $R
TAIL=$(python -c "import json,sys; print(json.load(open(sys.argv[1]))['overlay']['rounds_drained'])" $O/bench.json)
python profiles/steady_kernels.py $(find $O/trace -name "*kernel_trace.csv" | head -1) --steps ${STEPS:-20} --tail $TAIL --per-round > $O/steady.txt && cat $O/steady.txt
gzip -f $(find $O/trace -name "*kernel_trace.csv")
