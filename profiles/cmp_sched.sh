#!/bin/bash
# Config C under both schedules (survey = SURVEY 8(d), doubling = round 2's
# line), no CPU baseline.  Usage (repo root): bash profiles/cmp_sched.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for s in survey doubling; do
  timeout -k 10 300 python -u bench.py --schedule $s --no-cpu-baseline > $O/bench_$s.json 2> $O/$s.err || { echo $s FAILED; tail -5 $O/$s.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$s.json')); r=d['roofline']; print('$s', '%.4g' % d['value'], '%.4g msgs/s' % d['msgs_per_sec'], round(d['ms_per_step'],3), 'ms/step phase', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],4), 'step_frac', round(r['step_frac'],4), 'ovf', d['overflow'], 'rel', round(d['overlay']['tracked_broadcast_reliability'],5), 'hop', d['overlay']['tracked_broadcast_last_hop'])"
done
