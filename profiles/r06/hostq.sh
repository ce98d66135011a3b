#!/bin/bash
# Host enqueue time against GPU time per batch: the rank path and the local
# path, PSIM_TRACE_BATCH.  Usage: bash profiles/r06/hostq.sh TAG
TAG=${1:-r6hq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
PSIM_TRACE_BATCH=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rank-path --no-cpu-baseline --no-check > $O/bench_rank.json 2> $O/bench_rank.err || { tail -5 $O/bench_rank.err; exit 1; }
grep "batch of" $O/bench_rank.err | tail -8
PSIM_TRACE_BATCH=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-check > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
grep "batch of" $O/bench.err | tail -6
python3 -c "
import json
for f in ('$O/bench_rank.json', '$O/bench.json'):
    d = json.load(open(f)); print(f.split('/')[-1], round(d['ms_per_step'], 4), round(d['roofline']['avg_launch_ms'], 4))"
