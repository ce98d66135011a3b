#!/bin/bash
# Config E at its full 2^26 nodes on the box: the per-round attribution
# (profiles/e_attrib.py, phase timers) and the bench line under a rocprofv3
# kernel trace.  Usage (repo root): bash profiles/e26.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
PSIM_TRACE_GROW=1 timeout -k 10 600 python -u profiles/e_attrib.py --nodes 67108864 > $O/attrib.txt 2>&1 || { echo ATTRIB FAILED; tail -5 $O/attrib.txt; exit 1; }
tail -1 $O/attrib.txt
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u bench.py --workload E --nodes 67108864 --steps 60 --warmup 5 --no-cpu-baseline > $O/bench_E26.json 2> $O/E26.err || { echo E26 FAILED; tail -5 $O/E26.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_E26.json')); r=d['roofline']; print('E26', '%.3g' % d['value'], round(d['ms_per_step'],2), 'ms/step phase', round(r['avg_launch_ms'],2), 'frac', round(r['frac'],4), 'step_frac', round(r['step_frac'],4), 'ovf', d['overflow'])"
