#!/bin/bash
# Config E at 2^26 nodes under a kernel trace: per-round time by kernel over
# the 60-round window (profiles/round_kernels.py).  Usage (repo root): bash profiles/e26_trace.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 1000 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- \
  python3 -u $R/profiles/e_attrib.py --nodes 67108864 > $O/trace_attrib.txt 2>&1 || { echo TRACE FAILED; tail -5 $O/trace_attrib.txt; exit 1; }
T=$(find $O/tr -name "*kernel_trace.csv" | head -1)
cp $T $O/kernel_trace.csv && rm -rf $O/tr
python3 $R/profiles/round_kernels.py $O/kernel_trace.csv 60 > $O/e26_kernels.txt && cat $O/e26_kernels.txt
