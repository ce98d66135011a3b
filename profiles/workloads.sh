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
# config D's size (2^24 nodes) on one GPU: the HyParView+Plumtree overlay
# and the SCAMP v2 overlay it is compared with
timeout -k 10 400 python bench.py --nodes 16777216 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_C16M.json 2> $O/C16.err || { echo C16M FAILED; tail -5 $O/C16.err; exit 1; }
timeout -k 10 400 python bench.py --workload D --nodes 16777216 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_D16M.json 2> $O/D16.err || { echo D16M FAILED; tail -5 $O/D16.err; exit 1; }
for w in B D E_slice C16M D16M; do python -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', '%.3g' % d['value'], d['unit'], round(d['ms_per_step'],3), 'ms/step', 'frac', round(d['roofline']['frac'],4), 'ovf', d.get('overflow'))"; done
