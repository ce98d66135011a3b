#!/bin/bash
# Per-round work-list sizes of the node-round kernels (PSIM_TRACE_RELAY), a
# short bench window.  Usage (GPU box, repo root): bash profiles/trace_counts.sh TAG
O=gpurun_out/${1:-counts}; mkdir -p $O
PSIM_TRACE_RELAY=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-check > $O/bench.json 2> $O/trace.err || exit 1
grep "psim: round" $O/trace.err | tail -20
