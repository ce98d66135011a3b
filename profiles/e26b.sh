#!/bin/bash
# Config E at its full 2^26 nodes (SURVEY 8(d) schedule), the 140-round
# window of round 4's E26 line (--steps 140 --warmup 5), under a rocprofv3
# kernel trace; the per-kernel table of the timed rounds.
# Usage (repo root on the box): bash profiles/e26b.sh TAG [extra bench args]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u $R/bench.py --workload E --nodes 67108864 --steps 140 --warmup 5 --no-cpu-baseline "$@" > $O/bench_E26.json 2> $O/E26.err || { echo E26 FAILED; tail -5 $O/E26.err; exit 1; }
cd $R
python3 -c "import json; d=json.load(open('$O/bench_E26.json')); r=d['roofline']; print('E26', '%.3g' % d['value'], round(d['ms_per_step'],2), 'ms/step phase', round(r['avg_launch_ms'],2), 'frac', round(r['frac'],4), 'step_frac', round(r['step_frac'],4), 'ovf', d['overflow_run'])"
TAIL=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['overlay']['rounds_drained'])" $O/bench_E26.json)
python3 profiles/steady_kernels.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --steps 140 --tail $TAIL > $O/kernels.txt && head -30 $O/kernels.txt
gzip -f $(find $O/prof -name "*kernel_trace.csv")
