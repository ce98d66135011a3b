#!/bin/bash
# A/B of the lite list's kernel on the survey line: k_lite_half (default)
# against the wave-per-node k_consume_lite (PSIM_LITE_WAVE=1), after the GPU
# parity suite.  Usage (GPU box, repo root): bash profiles/r04/ab_lite.sh TAG [pytest -k expr]
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "$K" > $OUT/tests.txt 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
fi
rc=$?
tail -5 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
for v in half wave; do
  if [ $v = wave ]; then export PSIM_LITE_WAVE=1; else unset PSIM_LITE_WAVE; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-check > $OUT/bench_$v.json 2> $OUT/bench_$v.err || exit 1
  python - $OUT/bench_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("%s: node-rounds/s %.4g  ms/step %.3f  node-round phase %.3f ms  frac %.4f" % (
    sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"]))
PY
done
