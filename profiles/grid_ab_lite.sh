#!/bin/bash
# k_consume_lite's block shape and grid on the driver's bench command: each
# (library variant, PSIM_LITE_GRID) pair's bench line (survey schedule,
# --steps 20 --warmup 5), and a kernel trace of each for k_consume_lite's
# own time.  Usage (repo root): bash profiles/grid_ab_lite.sh TAG VARIANT:GRID ...
# (VARIANT "base" = libpartisan_gpu_sim.so; GRID 0 = the resident grid)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for vg in "$@"; do
  v=${vg%%:*}; g=${vg##*:}
  if [ "$v" = base ]; then L=""; else L=$v; fi
  if [ "$g" = 0 ]; then unset PSIM_LITE_GRID; else export PSIM_LITE_GRID=$g; fi
  PSIM_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t_$v_$g -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-check --steps 20 --warmup 5 > $O/bench_${v}_$g.json 2> $O/bench_${v}_$g.err \
    || { echo "BENCH FAILED $v $g"; tail -5 $O/bench_${v}_$g.err; exit 1; }
  S=$(find $O/t_$v_$g -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv, json
d = json.load(open('$O/bench_${v}_$g.json'))
lite = [r for r in csv.DictReader(open('$S')) if 'k_consume_lite' in r['Name']]
print('$v grid $g', round(d['ms_per_step'], 3), 'ms/step phase', round(d['roofline']['avg_launch_ms'], 3),
      'lite avg us', round(float(lite[0]['AverageNs']) / 1e3, 1) if lite else None)"
  rm -rf $O/t_$v_$g
done
echo AB DONE
