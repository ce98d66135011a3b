#!/bin/bash
# k_relay's binned lists (k_ptl's by BROADCAST presence, the lite list by
# SHUFFLE terminals) against one list each, and a 12-entry k_ptl table: a
# parity subset, then the survey line and E at 2^26.
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "config_a or doubling or churn or star or bench_schedule or loopback or plumtree or knobs" > gpurun_out/ab3_tests.txt 2>&1; rc=$?; tail -2 gpurun_out/ab3_tests.txt; [ $rc -eq 0 ] || exit $rc
bash profiles/r04/ab_env.sh ab3 "base:" "ptlbin:PSIM_LIB=ptlbin" "nobin:PSIM_LIB=nobin" "c12:PSIM_LIB=c12" || exit 1
BENCH_ARGS="--workload E --schedule doubling --nodes 67108864 --steps 20 --warmup 5" bash profiles/r04/ab_env.sh ab3e "base:" "nobin:PSIM_LIB=nobin" "c12:PSIM_LIB=c12"
