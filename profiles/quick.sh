#!/bin/bash
# Quick GPU iteration: a parity subset, then the headline bench window
# (node-round phase ms).  Usage (GPU box, repo root): bash profiles/quick.sh TAG
TAG=${1:-q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "config_a or doubling or churn or star or variants or revert or crash or shard_count or multistep or histograms_delivery or 1m or multi_root" > $OUT/tests.txt 2>&1
rc=$?
tail -2 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-check > $OUT/bench.json 2> $OUT/bench.err || exit 1
python - $OUT/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("node-rounds/s %.4g  ms/step %.3f  node-round phase %.3f ms  frac %.4f  msgs/s %.4g" % (
    d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], d["msgs_per_sec"]))
PY
