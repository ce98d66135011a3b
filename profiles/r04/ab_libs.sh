#!/bin/bash
# The survey line's node-round phase for library variants (PSIM_LIB=name),
# interleaved twice.  Usage (GPU box, repo root): bash profiles/r04/ab_libs.sh TAG v1 v2 ...
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for pass in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then unset PSIM_LIB; else export PSIM_LIB=$v; fi
    timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} --no-cpu-baseline --no-check > $O/bench_${v}_$pass.json 2> $O/bench_${v}_$pass.err || { echo "bench $v failed"; tail -3 $O/bench_${v}_$pass.err; exit 1; }
    python - $O/bench_${v}_$pass.json $v $pass <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("%-8s pass %s: ms/step %.3f  phase %.3f ms  frac %.4f" % (sys.argv[2], sys.argv[3], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"]))
PY
  done
done
