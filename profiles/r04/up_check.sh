#!/bin/bash
# k_ptl's connection mask from k_node_prep's up-and-partition pairs: a parity
# subset, the survey line, and E at 2^26 (round 3's schedule, 60 rounds)
# under a kernel trace.  Usage (GPU box, repo root): bash profiles/r04/up_check.sh TAG
TAG=${1:-up}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "config_a or doubling or churn or star or bench_schedule or loopback or knobs or plumtree or shard" > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
bash profiles/r04/ab_env.sh $TAG "base:" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- \
  python3 -u $R/bench.py --no-cpu-baseline --no-check --workload E --schedule doubling --nodes 67108864 --steps 60 --warmup 5 \
  > $O/bench_E26d.json 2> $O/E26d.err || { echo "E26 FAILED"; tail -5 $O/E26d.err; exit 1; }
cd $R
python3 profiles/round_kernels.py $(find $O/tr -name "*kernel_trace.csv" | head -1) 60 --tail 40 > $O/kernels_E26d.txt; rm -rf $O/tr
head -8 $O/kernels_E26d.txt
