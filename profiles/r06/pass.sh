#!/bin/bash
# A round-6 pass on the current source: the whole -m gpu suite, the driver's
# bench command, the rank path's line, and E at 2^26 with the buffers'
# high-water marks traced.  Usage (GPU box, repo root): bash profiles/r06/pass.sh TAG [notests]
TAG=${1:-r6pass}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$2" != "notests" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
  tail -3 $O/gpu_tests.txt
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rank-path --no-cpu-baseline > $O/bench_rank.json 2> $O/bench_rank.err || { tail -5 $O/bench_rank.err; exit 1; }
python3 - $O <<'PY'
import json, sys
for f in ("bench.json", "bench_rank.json"):
    d = json.load(open(sys.argv[1] + "/" + f)); r = d["roofline"]
    print(f, "%.4g node-rounds/s  ms/step %.4f  phase %.4f  frac %.4f  step_frac %.4f" % (d["value"], d["ms_per_step"], r["avg_launch_ms"], r["frac"], r["step_frac"]), "kernels", {k: round(v, 4) for k, v in d["kernel_ms_per_step"].items()})
PY
PSIM_TRACE_BOUND=1 timeout -k 10 900 python -u bench.py --workload E --nodes 67108864 --steps 140 --warmup 5 --no-cpu-baseline --strict > $O/bench_E26.json 2> $O/E26.err || { echo E26 FAILED; tail -5 $O/E26.err; exit 1; }
grep "psim:" $O/E26.err | tail -12
python3 -c "import json; d=json.load(open('$O/bench_E26.json')); r=d['roofline']; print('E26', '%.3g' % d['value'], round(d['ms_per_step'],2), 'ms/step phase', round(r['avg_launch_ms'],2), 'mem', d['device_mem_used_gb'], 'ovf', d['overflow_run']['total'])"
echo PASS DONE
