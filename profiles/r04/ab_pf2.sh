#!/bin/bash
# k_ptl: the next node's rows issued before this node's emissions, on top of
# the register records (pf4: 4 records, 168 VGPRs; pf2: 2 records, 159)
# against the library (6 records, no prefetch): a parity subset on each,
# then E at 2^26 and the survey line.
for v in pf4 pf2; do
  PSIM_LIB=$v timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "config_a or churn or bench_schedule or plumtree or e_mini" > gpurun_out/abpf2_tests_$v.txt 2>&1; rc=$?; tail -1 gpurun_out/abpf2_tests_$v.txt; [ $rc -eq 0 ] || exit $rc
done
BENCH_ARGS="--workload E --schedule doubling --nodes 67108864 --steps 20 --warmup 5" bash profiles/r04/ab_env.sh abpf2e "base:" "pf4:PSIM_LIB=pf4" "pf2:PSIM_LIB=pf2" || exit 1
bash profiles/r04/ab_env.sh abpf2c "base:" "pf4:PSIM_LIB=pf4" "pf2:PSIM_LIB=pf2"
