#!/bin/bash
# The secondary lines on the current source, each with its PMC traffic
# record: E at 2^26 (the SURVEY schedule, --strict) under a kernel trace, and
# configs B and D.  Usage (GPU box, repo root): bash profiles/r06/lines.sh TAG
TAG=${1:-lines}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash profiles/e26b.sh $TAG/e26 --strict > $O/e26.txt 2>&1; head -3 $O/e26.txt
bash profiles/run_pmc.sh ${TAG}_E26 --workload E --nodes 67108864 --steps 140 --warmup 5 --strict --no-check | tail -1
for w in B D; do
  timeout -k 10 400 python bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -3 $O/bench_$w.err; exit 1; }
  bash profiles/run_pmc.sh ${TAG}_$w --workload $w | tail -1
done
echo LINES DONE
