#!/bin/bash
# One iteration on k_lite_half: the lockstep record diff against the wave
# kernel, a parity subset, the A/B bench, then the kernel trace + SQ table.
# Usage (GPU box, repo root): bash profiles/r04/lite_iter.sh TAG [noprof]
TAG=${1:-it}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tests/_lite_diff2.py e_miniature > $O/diff.txt 2>&1; rc=$?
tail -3 $O/diff.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tests/_lite_diff2.py churn_partition > $O/diff2.txt 2>&1; rc=$?
tail -3 $O/diff2.txt
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/ab_lite.sh $TAG "config_a or doubling or churn or star or variants or 64k or bench_schedule or bucket or xbot or loopback" || exit 1
[ "$2" = "noprof" ] && exit 0
bash profiles/r04/prof_lite.sh $TAG
