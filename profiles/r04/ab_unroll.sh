#!/bin/bash
# k_ptl's LDS set scans unrolled (the library, PSIM_PTL_UNROLL=1) against
# runtime loops (u0) and the outstanding table's unrolled too (u3): a parity
# subset, then E at 2^26 and the survey line.
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "config_a or doubling or churn or star or bench_schedule or plumtree or knobs or xbot or e_mini" > gpurun_out/abu_tests.txt 2>&1; rc=$?; tail -2 gpurun_out/abu_tests.txt; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--workload E --schedule doubling --nodes 67108864 --steps 20 --warmup 5" bash profiles/r04/ab_env.sh abue "u1:" "u0:PSIM_LIB=u0" "u3:PSIM_LIB=u3" || exit 1
bash profiles/r04/ab_env.sh abuc "u1:" "u0:PSIM_LIB=u0" "u3:PSIM_LIB=u3"
