#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (profiles/calib/calib_fetch.hip), each
# counter its own pass.  Usage (GPU box, repo root): bash profiles/calib/run_calib.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/calib
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $R/profiles/calib/calib_fetch > $O/plain.txt || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $R/profiles/calib/calib_fetch > $O/fetch.txt 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $R/profiles/calib/calib_fetch > $O/write.txt 2>&1 || exit 1
cat $O/plain.txt
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for name in ("fetch", "write"):
    f = glob.glob(f"{o}/{name}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(f"{name:5s} {k:12s} per dispatch (KiB as reported): " + " ".join(f"{x:.0f}" for x in v))
PY
