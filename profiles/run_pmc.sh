#!/bin/bash
# HBM traffic of the node-round kernels for ONE bench.py command: a
# FETCH_SIZE pass and a WRITE_SIZE pass (each its own run: rocprofv3 does not
# split counters over passes), then profiles/pmc_record.py files the record
# under the command's pmc_key in profiles/pmc_records.json (copied back via
# gpurun_out/).  Usage (GPU box, repo root):
#   bash profiles/run_pmc.sh TAG [bench args, e.g. --steps 20 --warmup 5]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "k_relay|k_shuf|k_consume|k_lite|k_term|k_pt" -d $OUT/$c -o run \
    --output-format csv -- python3 $R/bench.py --no-cpu-baseline --kernel-counts "$@" > $OUT/$c.json 2> $OUT/$c.err \
    || { echo "$c pass failed"; tail -3 $OUT/$c.err; exit 1; }
done
cd $R
python3 profiles/pmc_record.py $OUT/FETCH_SIZE.json $(find $OUT/FETCH_SIZE -name "*counter_collection.csv" | head -1) \
  $(find $OUT/WRITE_SIZE -name "*counter_collection.csv" | head -1) > $OUT/record.json || exit 1
cp profiles/pmc_records.json $OUT/pmc_records.json
cat $OUT/record.json
rm -rf $OUT/FETCH_SIZE $OUT/WRITE_SIZE
