#!/bin/bash
# One measurement pass (GPU box, repo root): the GPU test suite, config C
# under both schedules, a kernel trace of the survey line (per-round kernel
# table and host gaps), then config E at 2^26.
# Usage: bash profiles/r03_pass2.sh TAG [skip-e26]
set -o pipefail
TAG=${1:-p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -4 $O/gpu_tests.log
[ $rc -le 1 ] || { echo "TESTS ABORTED rc=$rc"; exit 1; }
bash profiles/cmp_sched.sh $TAG/cmp || exit 1
STEPS=50 bash profiles/prof_steady.sh $TAG/steady_survey > /dev/null || exit 1
gunzip -k $(find $O/steady_survey/trace -name "*kernel_trace.csv.gz" | head -1) 2>/dev/null
F=$(find $O/steady_survey/trace -name "*kernel_trace.csv" | head -1)
python profiles/per_round.py $F 50 --tail $(python -c "import json,sys; print(json.load(open(sys.argv[1]))['overlay']['rounds_drained'])" $O/steady_survey/bench.json) > $O/steady_survey/per_round.txt
python profiles/gaps.py $F --steps 50 > $O/steady_survey/gaps.txt
rm -f $F
head -30 $O/steady_survey/steady.txt; tail -1 $O/steady_survey/per_round.txt; tail -12 $O/steady_survey/gaps.txt
[ "$2" = "skip-e26" ] && exit 0
bash profiles/e26.sh $TAG/e26 || exit 1
