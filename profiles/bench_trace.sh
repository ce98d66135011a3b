#!/bin/bash
# The driver's bench command under a kernel trace: per-round time by kernel
# over the timed window (profiles/round_kernels.py).
# Usage (repo root): bash profiles/bench_trace.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-check --steps 20 --warmup 5 "$@" > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -5 $O/bench.err; exit 1; }
T=$(find $O/tr -name "*kernel_trace.csv" | head -1)
cp $T $O/kernel_trace.csv && rm -rf $O/tr
D=$(python3 -c "import json; print(json.load(open('$O/bench.json'))['overlay']['rounds_drained'])")
python3 $R/profiles/round_kernels.py $O/kernel_trace.csv 20 --tail $D > $O/round_kernels.txt && cat $O/round_kernels.txt
