#!/bin/bash
# A/B on one box: a GPU parity subset on the current library, the driver's
# command for each C variant interleaved (profiles/abn.sh), then E at 2^26
# (SURVEY schedule, --strict) once per E variant.
# Usage: bash profiles/r06/ab2.sh TAG ROUNDS "C VARIANTS" "E VARIANTS"
# (a variant: base, NAME=VALUE[,NAME=VALUE..] on the base library, or the
# name of libpartisan_gpu_sim_<name>.so)
TAG=$1; ROUNDS=$2; CV=$3; EV=$4
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "config_a or doubling or churn or star or route_regrow or batch_regrow or bench_schedule or e_miniature or snapshot" > $O/parity.txt 2>&1; rc=$?
tail -2 $O/parity.txt
[ $rc -eq 0 ] || exit $rc
if [ -n "$CV" ]; then bash profiles/abn.sh $TAG $ROUNDS $CV || exit 1; fi
for v in $EV; do
  E=""
  if [ "$v" = base ]; then L=""; elif [[ "$v" == *=* ]]; then L=""; E=${v//,/ }; else L=$v; fi
  env $E PSIM_LIB=$L timeout -k 10 600 python -u bench.py --workload E --nodes 67108864 --steps 140 --warmup 5 \
      --no-cpu-baseline --strict > $O/e26_$v.json 2> $O/e26_$v.err || { echo "E26 FAILED $v"; tail -5 $O/e26_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e26_$v.json')); r=d['roofline']; print('E26 $v', '%.4g' % d['value'], round(d['ms_per_step'],3), 'ms/step phase', round(r['avg_launch_ms'],3), 'mem', d['device_mem_used_gb'], 'ovf', d['overflow_run']['total'])"
done
echo AB2 DONE
