#!/bin/bash
# Config E at 2^26 (the survey schedule, --strict) with the buffers'
# high-water marks traced (PSIM_TRACE_BOUND): the outbox bound and the routed
# record count against their reservations.
TAG=${1:-r6e26t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
PSIM_TRACE_BOUND=1 timeout -k 10 900 python -u bench.py --workload E --nodes 67108864 --steps 140 --warmup 5 --no-cpu-baseline --strict > $O/bench_E26.json 2> $O/E26.err || { echo E26 FAILED; tail -5 $O/E26.err; exit 1; }
grep "psim:" $O/E26.err | tail -20
python3 -c "import json; d=json.load(open('$O/bench_E26.json')); r=d['roofline']; print('E26', '%.3g' % d['value'], round(d['ms_per_step'],2), 'ms/step phase', round(r['avg_launch_ms'],2), 'mem', d['device_mem_used_gb'], 'ovf', d['overflow_run']['total'])"
