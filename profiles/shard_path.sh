#!/bin/bash
# The sharded round path on one GPU: G virtual shards (partition, device-copy
# exchange, receive route) against one shard of the same total size.
# Usage: bash profiles/shard_path.sh [TAG]
set -o pipefail
TAG=${1:-shard}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline --nodes $((1 << 21)) > $O/g1_2m.json 2> $O/g1.err || { echo G1 FAILED; tail $O/g1.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --vshards 2 > $O/g2_2m.json 2> $O/g2.err || { echo G2 FAILED; tail $O/g2.err; exit 1; }
PSIM_PHASE_TIMERS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --vshards 2 > $O/g2_phases.json 2> $O/g2p.err || { echo G2P FAILED; tail $O/g2p.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --vshards 2 > $O/g2_prof.json 2> $O/prof.err || { echo PROF FAILED; tail -20 $O/prof.err; exit 1; }
for f in $O/*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"; done
echo ALL DONE
