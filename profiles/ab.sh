#!/bin/bash
# A/B of library variants on the box: parity tests against each variant, then
# the bench line of each.  Usage: bash profiles/ab.sh TAG VARIANT...
# ("base" = libpartisan_gpu_sim.so, else libpartisan_gpu_sim_<VARIANT>.so)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L=$v; fi
  PSIM_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "TESTS FAILED $v"; tail -20 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
  PSIM_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { echo "BENCH FAILED $v"; tail -20 $O/bench_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$v.json')); print('$v', round(d['value']/1e6,1), 'M node-rounds/s', round(d['ms_per_step'],3), 'ms/step consume', round(d['kernel_ms_per_step']['consume'],3), 'frac', round(d['roofline']['frac'],4))"
done
echo AB DONE
