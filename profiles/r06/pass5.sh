#!/bin/bash
# The whole -m gpu suite on the current library, then C variants interleaved
# (profiles/abn.sh) and E at 2^26 (--strict) per E variant, the base one with
# the outbox and route high-water marks traced (PSIM_TRACE_BOUND).
# Usage (GPU box, repo root): bash profiles/r06/pass5.sh TAG ROUNDS "C VARIANTS" "E VARIANTS"
TAG=$1; ROUNDS=$2; CV=$3; EV=$4
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
if [ -n "$CV" ]; then bash profiles/abn.sh $TAG $ROUNDS $CV || exit 1; fi
for v in $EV; do
  E=""
  if [ "$v" = base ]; then L=""; E="PSIM_TRACE_BOUND=1"; elif [[ "$v" == *=* ]]; then L=""; E=${v//,/ }; else L=$v; fi
  env $E PSIM_LIB=$L timeout -k 10 600 python -u bench.py --workload E --nodes 67108864 --steps 140 --warmup 5 \
      --no-cpu-baseline --strict > $O/e26_$v.json 2> $O/e26_$v.err || { echo "E26 FAILED $v"; tail -5 $O/e26_$v.err; exit 1; }
  grep "outbox total max" $O/e26_$v.err | tail -1
  python3 -c "import json; d=json.load(open('$O/e26_$v.json')); r=d['roofline']; print('E26 $v', '%.4g' % d['value'], round(d['ms_per_step'],3), 'ms/step phase', round(r['avg_launch_ms'],3), 'mem', d['device_mem_used_gb'], 'ovf', d['overflow_run']['total'])"
done
echo PASS5 DONE
