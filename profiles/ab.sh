#!/bin/bash
# A/B of library variants on one box: bash profiles/ab.sh OUT lib1 lib2 ...
# (each lib under build/variants/, copied over the in-tree library in turn)
OUT=$1; shift
mkdir -p gpurun_out
L=partisan_amd/csrc/libpartisan_gpu_sim.so
cp $L /tmp/psim_orig.so
for v in "$@"; do
    cp build/variants/$v.so $L
    if [[ $v == *stamps* ]]; then
        timeout -k 10 200 python profiles/stamps.py > gpurun_out/${OUT}_$v.txt 2>&1 || exit 1
    else
        timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline > gpurun_out/${OUT}_$v.json 2>gpurun_out/${OUT}_$v.err || exit 1
    fi
done
cp /tmp/psim_orig.so $L
