#!/bin/bash
O=gpurun_out/${1:-diag1}; mkdir -p $O
PSIM_TRACE_RELAY=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-check > $O/bench_trace.json 2> $O/trace.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-check > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/prof.err || exit 1
gzip -f $GRAFT_REPO_ROOT/$O/prof/run_kernel_trace.csv
echo done
