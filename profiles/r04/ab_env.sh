#!/bin/bash
# The survey line's node-round phase under environment variants, interleaved
# twice.  Usage (GPU box, repo root): bash profiles/r04/ab_env.sh TAG "NAME:VAR=V VAR2=V2" ...
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for pass in 1 2; do
  for spec in "$@"; do
    name=${spec%%:*}; vars=${spec#*:}
    [ "$vars" = "$spec" ] && vars=""
    timeout -k 10 300 env $vars python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} --no-cpu-baseline --no-check > $O/bench_${name}_$pass.json 2> $O/bench_${name}_$pass.err || { echo "bench $name failed"; tail -3 $O/bench_${name}_$pass.err; exit 1; }
    python - $O/bench_${name}_$pass.json $name $pass <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("%-10s pass %s: ms/step %.3f  phase %.3f ms  frac %.4f" % (sys.argv[2], sys.argv[3], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"]))
PY
  done
done
