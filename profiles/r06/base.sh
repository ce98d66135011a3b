#!/bin/bash
# Round-6 first pass: the -m gpu suite and the driver's bench command.
TAG=${1:-r6base}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
cat $O/bench.json | head -c 600
