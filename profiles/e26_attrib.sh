#!/bin/bash
# Config E at its full 2^26 nodes, the per-round attribution (phase timers,
# buffer growth traced): profiles/e_attrib.py.  Usage (repo root): bash profiles/e26_attrib.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
PSIM_TRACE_GROW=1 timeout -k 10 1000 python -u profiles/e_attrib.py --nodes 67108864 > $O/attrib.txt 2>&1 || { echo ATTRIB FAILED; tail -5 $O/attrib.txt; exit 1; }
grep -c "psim: grow" $O/attrib.txt; tail -3 $O/attrib.txt
