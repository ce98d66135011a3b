#!/bin/bash
# SQ/TCC counter passes over bench.py (one pass per counter group; each pass
# its own run, as rocprofv3 does not split counters over passes).
# Usage (GPU box, repo root): bash profiles/run_pmc.sh TAG [bench args]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
pass() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 3 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }
}
pass p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
pass p2 SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC
pass p3 FETCH_SIZE
pass p4 WRITE_SIZE
python3 $R/profiles/pmc_summary.py $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 --rounds 10 > $OUT/summary.txt
cat $OUT/summary.txt
rm -rf $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4      # keep gpurun_out small (<64 MiB merges back)
echo pmc done
