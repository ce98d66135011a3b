#!/bin/bash
# k_ptl without the LDS copy of the slot table (PSIM_LIB=nosl: 14488 B of
# LDS a block, 11 blocks per CU instead of 10) against the library: a parity
# subset on the variant, then E at 2^26 and the survey line.
PSIM_LIB=nosl timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "config_a or doubling or churn or star or bench_schedule or plumtree or xbot or e_mini" > gpurun_out/absl_tests.txt 2>&1; rc=$?; tail -2 gpurun_out/absl_tests.txt; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--workload E --schedule doubling --nodes 67108864 --steps 20 --warmup 5" bash profiles/r04/ab_env.sh absle "base:" "nosl:PSIM_LIB=nosl" || exit 1
bash profiles/r04/ab_env.sh abslc "base:" "nosl:PSIM_LIB=nosl"
