#!/bin/bash
# Host-trap PC sampling of the driver's bench command, samples of the
# node-round kernels only (profiles/pcs_hot.py maps them to source lines).
# Usage (GPU box, repo root): bash profiles/pcs_lite.sh TAG [INTERVAL_US]
set -o pipefail
TAG=${1:-pcs}
IV=${2:-20}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval $IV -d $O/pcs -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-check \
  --steps 20 --warmup 5 > $O/bench.json 2> $O/pcs.err || { echo PCS FAILED; tail -20 $O/pcs.err; exit 1; }
ls -la $(find $O/pcs -type f) | head
for f in $(find $O/pcs -name "*.csv"); do head -3 $f; wc -l $f; done
gzip -f $(find $O/pcs -name "*.csv")
echo PCS DONE
