#!/bin/bash
# Quick A/B of library variants (bench only, alternating, twice each):
# node-round phase ms per variant.  Parity of the winner is run separately.
# Usage (GPU box): bash profiles/abq.sh TAG VARIANT...  ("base" = the product library)
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L=$v; fi
    PSIM_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --steps 20 --warmup 5 > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || { echo "BENCH FAILED $v"; tail -5 $O/b_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b_${v}_$rep.json')); print('$v', $rep, 'ms/step %.3f node-round %.3f ms' % (d['ms_per_step'], d['roofline']['avg_launch_ms']))"
  done
done
