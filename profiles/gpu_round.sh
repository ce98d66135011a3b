#!/bin/bash
# One GPU session on the box (run from the repo root through gpurun):
# parity tests, the default bench line, a rocprofv3 kernel-trace summary of
# the same bench command, and the per-phase stamps of k_consume.
# Usage: bash profiles/gpu_round.sh [TAG]
set -o pipefail
TAG=${1:-cur}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/prof.err || { echo PROF FAILED; tail -20 $O/prof.err; exit 1; }
cd $R
if [ -f partisan_amd/csrc/libpartisan_gpu_sim_stamps.so ]; then
  PSIM_LIB=stamps timeout -k 10 200 python profiles/stamps.py > $O/stamps.txt 2>&1 || { echo STAMPS FAILED; tail -20 $O/stamps.txt; exit 1; }
  cat $O/stamps.txt
fi
echo ALL DONE
