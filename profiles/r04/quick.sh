#!/bin/bash
# A parity subset, the survey line twice and the k_lite_half stamps.
# Usage (GPU box, repo root): bash profiles/r04/quick.sh TAG [pytest -k expr]
TAG=${1:-q}
O=gpurun_out/$TAG
mkdir -p $O
K=${2:-"config_a or doubling or churn or star or bench_schedule or loopback or knobs or bucket"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/ab_env.sh $TAG "base:" || exit 1
PSIM_LIB=stamps timeout -k 10 300 python3 profiles/stamps.py --steps 20 > $O/stamps.txt 2>&1 && tail -11 $O/stamps.txt
