#!/bin/bash
# SQ counters (one pass) of the node-round kernels over a short bench run:
# wave cycles split into waiting (s_waitcnt), issue-stalled and active, plus
# instruction mix.  Usage (GPU box, repo root): bash profiles/sq_split.sh TAG
TAG=${1:-sq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  --kernel-include-regex "k_consume|k_pt|k_relay" -d $O/pmc -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-check --steps 10 --warmup 3 > $O/bench.json 2> $O/pmc.err || { echo "pmc failed"; tail -3 $O/pmc.err; exit 1; }
cd $R
D=$(dirname $(find $O/pmc -name "*counter_collection.csv" | head -1))
TAIL=$(python -c "import json,sys; print(json.load(open(sys.argv[1]))['overlay']['rounds_drained'])" $O/bench.json)
for k in "k_relay(" "k_consume(" "k_pt("; do python profiles/pmc_summary.py $D --kernels "$k" --rounds 10 --tail $TAIL; done > $O/sq.txt
cat $O/sq.txt
