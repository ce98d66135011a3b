#!/bin/bash
# The rank path after the batched fixed-size exchange: its parity tests, then
# bench.py --rank-path (one-rank RCCL communicator) against the local path.
TAG=${1:-r6rank}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_rccl1.py tests/test_loopback.py tests/test_gpu_knobs.py -x -q --timeout 300 --timeout-method thread > $O/rank_tests.txt 2>&1; rc=$?
tail -3 $O/rank_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rank-path --no-cpu-baseline > $O/bench_rank.json 2> $O/bench_rank.err || { tail -5 $O/bench_rank.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O <<'PY'
import json, sys
for f in ("bench_rank.json", "bench.json"):
    d = json.load(open(sys.argv[1] + "/" + f)); r = d["roofline"]
    print(f, "%.4g node-rounds/s  ms/step %.4f  phase %.4f  check %s  x %s" % (d["value"], d["ms_per_step"], r["avg_launch_ms"], d.get("check", {}).get("ok") if isinstance(d.get("check"), dict) else d.get("check"), d.get("exchange")))
PY
