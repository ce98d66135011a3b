#!/bin/bash
# SQ counter passes over bench.py (one pass per counter group).
# Usage (GPU box, repo root): bash profiles/run_pmc.sh TAG [bench args]
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/p1 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/b1.json 2> $OUT/p1.err || { echo p1 failed; tail -3 $OUT/p1.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/b2.json 2> $OUT/p2.err || { echo p2 failed; tail -3 $OUT/p2.err; exit 1; }
echo pmc done
