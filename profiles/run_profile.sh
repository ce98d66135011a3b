#!/bin/bash
# Collects the rocprofv3 kernel-trace summary and HBM counters of bench.py.
# Usage (on the GPU box, from the repo root): bash profiles/run_profile.sh TAG [bench args]
set -e
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/bench.json
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_fetch.json
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_write.json
echo profile done
