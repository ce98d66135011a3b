#!/bin/bash
# The round's measurement pass (GPU box, repo root, through gpurun): the GPU
# test suite, the default bench line (the driver's command) and the
# --steps 20 --warmup 5 line, a rocprofv3 kernel-trace summary of the default
# command, and PMC traffic records for both commands.
# Usage: bash profiles/round_end.sh TAG
set -o pipefail
TAG=${1:-end}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || { echo BENCH FAILED; tail -20 $O/bench_20_5.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/prof.err || { echo PROF FAILED; tail -20 $O/prof.err; exit 1; }
cd $R
find $O/prof -name "*kernel_trace.csv" -exec gzip -f {} \;
bash profiles/run_pmc.sh ${TAG}_50 || exit 1
bash profiles/run_pmc.sh ${TAG}_20 --steps 20 --warmup 5 || exit 1
cp profiles/pmc_records.json $O/pmc_records.json
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for f in ("bench.json", "bench_20_5.json"):
    d = json.load(open(f"{o}/{f}"))
    print(f, "value %.4g ms/step %.3f node-round %.3f frac %.4f" % (d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"]))
PY
echo ALL DONE
