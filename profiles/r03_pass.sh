#!/bin/bash
# One measurement pass of this session (GPU box, repo root): the GPU test
# suite, config C under both schedules, then config E at 2^26.
# Usage: bash profiles/r03_pass.sh TAG
set -o pipefail
TAG=${1:-p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash profiles/cmp_sched.sh $TAG/cmp || exit 1
bash profiles/e26.sh $TAG/e26 || exit 1
