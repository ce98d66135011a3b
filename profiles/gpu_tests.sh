#!/bin/bash
# The GPU test suite on the box (repo root), log under gpurun_out/TAG.
# Usage: bash profiles/gpu_tests.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${K[@]}" > $O/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/gpu_tests.log | tail -15
exit $rc
