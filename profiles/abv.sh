#!/bin/bash
# Parity subset for each library variant, then the interleaved A/B bench
# (profiles/abn.sh).  Usage: bash profiles/abv.sh TAG ROUNDS VARIANT...
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for v in "$@"; do
  E=""
  if [ "$v" = base ]; then L=""; elif [[ "$v" == *=* ]]; then L=""; E=${v//,/ }; else L=$v; fi
  env $E PSIM_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "config_a or churn or star or 1m or bench_schedule or bucket_table or multi_root" > $O/tests_$v.log 2>&1 \
    || { echo "TESTS FAILED $v"; tail -5 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
bash $R/profiles/abn.sh $TAG $ROUNDS "$@"
