#!/bin/bash
# The whole -m gpu suite, then the default bench line.
# Usage (GPU box, repo root): bash profiles/r04/full.sh TAG
TAG=${1:-full}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -4 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
cat $O/bench.json
