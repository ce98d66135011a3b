#!/bin/bash
# Config E at 2^26 on SURVEY 8(d)'s schedule on the final source: the line
# under a kernel trace (--stats), its PMC traffic record, then the line again
# reading the record back.  Usage (GPU box, repo root): bash profiles/r04/e26_final.sh TAG
TAG=${1:-e26f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
E26S="--workload E --schedule survey --nodes 67108864 --steps 140 --warmup 5"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- \
  python3 -u $R/bench.py --no-cpu-baseline --no-check $E26S > $O/bench_trace.json 2> $O/trace.err || { echo TRACE FAILED; tail -5 $O/trace.err; exit 1; }
cd $R
cp $(find $O/tr -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
python3 profiles/round_kernels.py $(find $O/tr -name "*kernel_trace.csv" | head -1) 140 --tail 40 > $O/kernels.txt; rm -rf $O/tr
head -9 $O/kernels.txt
bash profiles/run_pmc.sh ${TAG} $E26S --no-check | tail -1 || exit 1
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-check $E26S > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']; o=d['overlay']
print('E26s %.3g ms/step %.2f phase %.2f frac %.4f step_frac %.4f traffic %.4g rel %.5f comps %d ovf %d' % (d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['step_frac'], r['traffic'], o['tracked_broadcast_reliability'], o['components'], d['overflow']))"
