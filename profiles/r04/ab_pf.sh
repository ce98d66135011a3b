#!/bin/bash
# k_ptl with the next node's rows prefetched (the library) against without
# (PSIM_LIB=nopf): a parity subset, then E at 2^26 and the survey line.
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "config_a or doubling or churn or star or bench_schedule or plumtree or knobs or xbot or e_mini" > gpurun_out/abpf_tests.txt 2>&1; rc=$?; tail -2 gpurun_out/abpf_tests.txt; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--workload E --schedule doubling --nodes 67108864 --steps 20 --warmup 5" bash profiles/r04/ab_env.sh abpfe "pf:" "nopf:PSIM_LIB=nopf" || exit 1
bash profiles/r04/ab_env.sh abpfc "pf:" "nopf:PSIM_LIB=nopf"
