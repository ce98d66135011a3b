#!/bin/bash
# The non-headline bench lines (configs B, D and an E slice) on the box.
# Usage (repo root): bash profiles/workloads.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --workload B --no-cpu-baseline > $O/bench_B.json 2> $O/B.err || { echo B FAILED; tail -5 $O/B.err; exit 1; }
timeout -k 10 300 python bench.py --workload D --no-cpu-baseline > $O/bench_D.json 2> $O/D.err || { echo D FAILED; tail -5 $O/D.err; exit 1; }
timeout -k 10 400 python bench.py --workload E --nodes 8388608 --steps 60 --warmup 10 --no-cpu-baseline > $O/bench_E_slice.json 2> $O/E.err || { echo E FAILED; tail -5 $O/E.err; exit 1; }
for w in B D E_slice; do python -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', '%.3g' % d['value'], d['unit'], round(d['ms_per_step'],3), 'ms/step', 'frac', round(d['roofline']['frac'],4), 'ovf', d.get('overflow'))"; done
