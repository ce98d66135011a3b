#!/bin/bash
# Measurement pass of the driver's bench command (python3 bench.py --gpus 1
# --steps 20 --warmup 5) on the GPU box, repo root: the bench line, a kernel
# trace of the same command (per-round kernel table, host gaps), the SQ
# counters of the node-round kernels, and the FETCH/WRITE traffic record for
# the command's pmc_key (profiles/pmc_records.json).
# Usage: bash profiles/r03_meas.sh TAG [skip-pmc]
set -o pipefail
TAG=${1:-m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('bench', '%.4g' % d['value'], round(d['ms_per_step'],3), 'ms/step phase', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],4), 'step_frac', round(r['step_frac'],4), 'ovf', d['overflow'], 'cpu', d['cpu_baseline']['value'])"
STEPS=20 bash profiles/prof_steady.sh $TAG/steady > /dev/null || exit 1
gunzip -k $(find $O/steady/trace -name "*kernel_trace.csv.gz" | head -1) 2>/dev/null
F=$(find $O/steady/trace -name "*kernel_trace.csv" | head -1)
python profiles/per_round.py $F 20 --tail $(python -c "import json,sys; print(json.load(open(sys.argv[1]))['overlay']['rounds_drained'])" $O/steady/bench.json) > $O/steady/per_round.txt
python profiles/gaps.py $F --steps 20 > $O/steady/gaps.txt
python profiles/round_kernels.py $F 20 --tail $(python -c "import json,sys; print(json.load(open(sys.argv[1]))['overlay']['rounds_drained'])" $O/steady/bench.json) > $O/steady/round_kernels.txt
rm -f $F
tail -1 $O/steady/per_round.txt; head -12 $O/steady/steady.txt
bash profiles/sq_kernels.sh $TAG/sq --steps 20 --warmup 5 > /dev/null || exit 1
tail -12 $O/sq/sq_kernels.txt
[ "$2" = "skip-pmc" ] && exit 0
bash profiles/run_pmc.sh $TAG --gpus 1 --steps 20 --warmup 5 || exit 1
