#!/bin/bash
# Host-trap PC sampling of the default bench command (k_consume hot spots).
# Usage: bash profiles/pc_sample.sh [TAG] [INTERVAL_US]
set -o pipefail
TAG=${1:-pcs}
IV=${2:-50}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval $IV -d $O/pcs -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 \
  > $O/bench.json 2> $O/pcs.err || { echo PCS FAILED; tail -30 $O/pcs.err; exit 1; }
ls -la $O/pcs/* | head
echo PCS DONE
