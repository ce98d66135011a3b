#!/bin/bash
# Per-kernel SQ counters of the six node-round kernels over a short bench run
# (one rocprofv3 --pmc pass): wave cycles split into waiting / issuing,
# instruction mix, and the achieved occupancy
#   waves per SIMD = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)
# (SQ_WAVE_CYCLES counts quad-cycles summed over waves; GRBM_GUI_ACTIVE is
# the kernel's cycles summed over the 8 XCDs; 1024 SIMDs).
# Usage (GPU box, repo root): bash profiles/sq_kernels.sh TAG [bench args]
TAG=${1:-sq}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_consume|k_pt|k_relay|k_shuf|k_term|k_lite" -d $O/pmc -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-check "$@" > $O/bench.json 2> $O/pmc.err || { echo "pmc failed"; tail -3 $O/pmc.err; exit 1; }
cd $R
F=$(find $O/pmc -name "*counter_collection.csv" | head -1)
python3 profiles/sq_table.py $F $O/bench.json > $O/sq_kernels.txt && cat $O/sq_kernels.txt
gzip -f $F
