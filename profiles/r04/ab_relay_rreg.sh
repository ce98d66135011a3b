#!/bin/bash
# k_relay with its first records' type words and sources held in registers
# (rl2 / rl4; 96 VGPRs, 12 B spilled) against the library: a parity subset on
# rl4, then the survey line and E at 2^26.
PSIM_LIB=rl4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "config_a or doubling or churn or star or bench_schedule or e_mini" > gpurun_out/abrl_tests.txt 2>&1; rc=$?; tail -2 gpurun_out/abrl_tests.txt; [ $rc -eq 0 ] || exit $rc
bash profiles/r04/ab_env.sh abrlc "base:" "rl2:PSIM_LIB=rl2" "rl4:PSIM_LIB=rl4" || exit 1
BENCH_ARGS="--workload E --schedule doubling --nodes 67108864 --steps 20 --warmup 5" bash profiles/r04/ab_env.sh abrle "base:" "rl4:PSIM_LIB=rl4"
