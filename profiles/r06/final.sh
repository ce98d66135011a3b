#!/bin/bash
# The round-6 measurement pass of the headline line on the current source:
# the driver's command (bench.py --steps 20 --warmup 5, with the CPU
# baseline), its rocprofv3 --kernel-trace --stats summary, the SQ table, the
# PMC traffic record (FETCH_SIZE / WRITE_SIZE passes of that command), the
# stamps build's phase split, and the default bench line.
# Usage (GPU box, repo root): bash profiles/r06/final.sh TAG
TAG=${1:-fin}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]
print("bench %.4g node-rounds/s  ms/step %.4f  phase %.4f ms  frac %.4f  step_frac %.4f  rel %.5f" % (
    d["value"], d["ms_per_step"], r["avg_launch_ms"], r["frac"], r["step_frac"], d["overlay"]["tracked_broadcast_reliability"]))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-check --steps 20 --warmup 5 > $O/prof_bench.json 2> $O/prof.err || { echo PROF FAILED; tail -5 $O/prof.err; exit 1; }
cd $R
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
TAIL=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['overlay']['rounds_drained'])" $O/prof_bench.json)
python3 profiles/steady_kernels.py $T --steps 20 --tail $TAIL --per-round > $O/steady.txt && head -18 $O/steady.txt
gzip -c $T > $O/kernel_trace.csv.gz && rm -rf $O/prof
bash profiles/sq_kernels.sh $TAG/sq --steps 20 --warmup 5 > /dev/null || exit 1
tail -8 $O/sq/sq_kernels.txt
bash profiles/run_pmc.sh $TAG --steps 20 --warmup 5 --no-check | tail -1
[ -f partisan_amd/csrc/libpartisan_gpu_sim_stamps.so ] && PSIM_LIB=stamps timeout -k 10 300 python3 profiles/stamps.py --steps 20 > $O/stamps.txt 2>&1 && tail -12 $O/stamps.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -3 $O/bench_default.err; exit 1; }
echo ALL DONE
