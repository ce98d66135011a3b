#!/bin/bash
# Upper bound of k_ptl's member loads (the connection mask's up-and-partition
# pairs): the variant skips them (wrong results, --no-check), E at 2^26 and C.
BENCH_ARGS="--workload E --schedule doubling --nodes 67108864 --steps 20 --warmup 5" bash profiles/r04/ab_env.sh abne "base:" "noup:PSIM_LIB=noup" || exit 1
bash profiles/r04/ab_env.sh abnc "base:" "noup:PSIM_LIB=noup"
