#!/bin/bash
# A/B of library variants on one box, interleaved: the driver's headline
# command (--steps 20 --warmup 5, no CPU baseline, no check) for each
# variant in turn, ROUNDS times.  Usage: bash profiles/abn.sh TAG ROUNDS VARIANT...
# ("base" = libpartisan_gpu_sim.so, NAME=VALUE[,NAME=VALUE..] = the base
# library with those environment variables set, else
# libpartisan_gpu_sim_<VARIANT>.so)
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for k in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    E=""
    if [ "$v" = base ]; then L=""; elif [[ "$v" == *=* ]]; then L=""; E=${v//,/ }; else L=$v; fi
    env $E PSIM_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-check > $O/bench_${v}_$k.json 2> $O/bench_${v}_$k.err || { echo "BENCH FAILED $v"; tail -20 $O/bench_${v}_$k.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${v}_$k.json')); kt=d['kernel_ms_per_step']; print('$v', $k, '%.4g node-rounds/s' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'phase %.4f' % d['roofline']['avg_launch_ms'], 'frac %.4f' % d['roofline']['frac'], ' '.join('%s %.4f' % (k_, v_) for k_, v_ in sorted(kt.items()) if v_ > 0.002))"
  done
done
echo AB DONE
