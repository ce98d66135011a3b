#!/bin/bash
# The other bench lines on the final source (not the driver's headline):
# E at its full 2^26 nodes, B, D at 2^21, C (survey schedule) at 2^24.
# Usage (repo root): bash profiles/r03_lines.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
line() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > $O/bench_$n.json 2> $O/$n.err || { echo "$n FAILED"; tail -5 $O/$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$n.json')); r=d['roofline']; print('$n', '%.3g' % d['value'], round(d['ms_per_step'],3), 'ms/step frac', round(r['frac'],4), 'step_frac', round(r.get('step_frac', 0) or 0,4), 'ovf', d['overflow'])"
}
line E26 --workload E --nodes 67108864 --steps 60 --warmup 5
line C24 --nodes 16777216 --steps 20 --warmup 5
line B --workload B --steps 20 --warmup 5
line D21 --workload D --steps 20 --warmup 5
