#!/bin/bash
# Kernel trace + SQ counters of the survey line with k_lite_half, and the SQ
# counters with the wave kernel (PSIM_LITE_WAVE=1) beside it.
# Usage (GPU box, repo root): bash profiles/r04/prof_lite.sh TAG
TAG=${1:-pl}
STEPS=20 bash profiles/prof_steady.sh $TAG/steady > /dev/null || exit 1
head -14 gpurun_out/$TAG/steady/steady.txt
bash profiles/sq_kernels.sh $TAG/sq_half --steps 20 --warmup 5 > /dev/null || exit 1
tail -9 gpurun_out/$TAG/sq_half/sq_kernels.txt
PSIM_LITE_WAVE=1 bash profiles/sq_kernels.sh $TAG/sq_wave --steps 20 --warmup 5 > /dev/null || exit 1
tail -9 gpurun_out/$TAG/sq_wave/sq_kernels.txt
