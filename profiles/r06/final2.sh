#!/bin/bash
# The last round-6 measurement pass on the final source: the headline's
# records (final.sh: bench, rocprofv3 kernel table, SQ, PMC, stamps, default
# line) and the rank path's line.  Usage (GPU box, repo root):
#   bash profiles/r06/final2.sh TAG
TAG=${1:-fin2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
cd $R
bash profiles/r06/final.sh $TAG || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rank-path --no-cpu-baseline > $O/bench_rank.json 2> $O/bench_rank.err || { tail -5 $O/bench_rank.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_rank.json')); print('rank', '%.4g' % d['value'], round(d['ms_per_step'], 4), 'ms/step')"
echo FINAL2 DONE
