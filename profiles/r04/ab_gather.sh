#!/bin/bash
# k_gather_dev variants (engine TU): g1 two quarters per lane a step, g2 one
# record per lane (four 16-B loads in flight) against the library's four
# lanes per record: a parity subset on each, then E at 2^26 and the survey line.
for v in g1 g2; do
  PSIM_LIB=$v timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "config_a or churn or bench_schedule or e_mini" > gpurun_out/abg_tests_$v.txt 2>&1; rc=$?; tail -1 gpurun_out/abg_tests_$v.txt; [ $rc -eq 0 ] || exit $rc
done
BENCH_ARGS="--workload E --schedule doubling --nodes 67108864 --steps 20 --warmup 5" bash profiles/r04/ab_env.sh abge "base:" "g1:PSIM_LIB=g1" "g2:PSIM_LIB=g2" || exit 1
bash profiles/r04/ab_env.sh abgc "base:" "g1:PSIM_LIB=g1" "g2:PSIM_LIB=g2"
