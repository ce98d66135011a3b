#!/bin/bash
# k_ptl with its first Plumtree records kept in registers from the
# precondition pass (PSIM_PTL_RREG: 4 in the library; r0 / r2 / r6 variants):
# the full parity suite, then E at 2^26 and the survey line.
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abr_tests.txt 2>&1; rc=$?; tail -2 gpurun_out/abr_tests.txt; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--workload E --schedule doubling --nodes 67108864 --steps 20 --warmup 5" bash profiles/r04/ab_env.sh abre "r4:" "r0:PSIM_LIB=r0" "r2:PSIM_LIB=r2" "r6:PSIM_LIB=r6" || exit 1
bash profiles/r04/ab_env.sh abrc "r4:" "r0:PSIM_LIB=r0" "r2:PSIM_LIB=r2" "r6:PSIM_LIB=r6"
