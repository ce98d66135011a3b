#!/bin/bash
# The rank path's parity tests (RCCL one-rank, loopback, knobs), then its
# line under a kernel trace (profiles/r06/ranktrace.sh).
TAG=${1:-r6rk}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_rccl1.py tests/test_loopback.py tests/test_gpu_knobs.py -x -q --timeout 300 --timeout-method thread > $O/rank_tests.txt 2>&1; rc=$?
tail -3 $O/rank_tests.txt
[ $rc -eq 0 ] || exit $rc
bash profiles/r06/ranktrace.sh $TAG
