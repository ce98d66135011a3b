#!/bin/bash
# Grids (and library variants) of the node-round kernels on the driver's bench
# command (survey schedule, --steps 20 --warmup 5): per entry the bench line
# and, from a kernel trace, each node-round kernel's average time.
# Usage (repo root): bash profiles/grid_ab.sh TAG ENTRY ...
#   ENTRY = VARIANT[:NAME=VALUE[,NAME=VALUE...]], VARIANT "base" =
#   libpartisan_gpu_sim.so, NAME e.g. PSIM_LITE_GRID, PSIM_PTL_GRID,
#   PSIM_PT_GRID, PSIM_CONSUME_GRID;
#   VALUE = blocks, or xK = K times the resident grid
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
k=0
for e in "$@"; do
  k=$((k + 1))
  v=${e%%:*}; envs=""
  [ "$e" != "$v" ] && envs=${e#*:}
  if [ "$v" = base ]; then L=""; else L=$v; fi
  ( export PSIM_LIB=$L; IFS=','; for kv in $envs; do export "$kv"; done
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t$k -o run --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --no-check --steps 20 --warmup 5 > $O/bench_$k.json 2> $O/bench_$k.err ) \
    || { echo "BENCH FAILED $e"; tail -5 $O/bench_$k.err; exit 1; }
  S=$(find $O/t$k -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv, json
d = json.load(open('$O/bench_$k.json'))
ks = {r['Name']: float(r['AverageNs']) / 1e3 for r in csv.DictReader(open('$S'))}
pick = lambda s: next((round(v, 1) for n, v in ks.items() if s in n), None)
print('$e', round(d['ms_per_step'], 3), 'ms/step phase', round(d['roofline']['avg_launch_ms'], 3),
      'lite', pick('k_consume_lite'), 'ptl', pick('k_ptl('), 'pt', pick('k_pt('), 'relay', pick('k_relay'), 'cons', pick('k_consume('),
      '| hist', pick('k_bucket_hist'), 'scat', pick('k_bucket_scatter'), 'route', pick('k_bucket_route'), 'gath', pick('k_gather'))" | tee -a $O/ab.txt
  rm -rf $O/t$k
done
echo AB DONE
