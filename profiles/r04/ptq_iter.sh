#!/bin/bash
# One iteration on k_ptq: a parity subset of the GPU tests, then the survey
# line and config E at 2^26 with k_ptq (base), its occupancy variants and
# k_ptl (PSIM_PTL_LANE=1).  Usage (GPU box, repo root): bash profiles/r04/ptq_iter.sh TAG [noe26]
TAG=${1:-pq}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "config_a or doubling or churn or star or variants or 64k or bench_schedule or bucket or loopback or plumtree or e_overlay" \
  > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/ab_env.sh $TAG "ptq:" "q4:PSIM_LIB=q4" "q6:PSIM_LIB=q6" "ptl:PSIM_PTL_LANE=1" || exit 1
[ "$2" = "noe26" ] && exit 0
BENCH_ARGS="--workload E --schedule doubling --nodes 67108864 --steps 20 --warmup 5" \
  bash profiles/r04/ab_env.sh ${TAG}e "ptq:" "q4:PSIM_LIB=q4" "ptl:PSIM_PTL_LANE=1"
