#!/bin/bash
# A/B on one box: a GPU parity subset on the current library, then the
# driver's command for each variant, interleaved (profiles/abn.sh).
# Usage: bash profiles/r06/ab.sh TAG ROUNDS VARIANT...
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "config_a or doubling or churn or star or route_regrow or batch_regrow or bench_schedule or e_miniature or snapshot" > $O/parity.txt 2>&1; rc=$?
tail -2 $O/parity.txt
[ $rc -eq 0 ] || exit $rc
bash profiles/abn.sh $TAG "$@"
