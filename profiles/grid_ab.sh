O=gpurun_out/ab_grid; mkdir -p $O
for rep in 1 2; do for g in 0 2048 1792 1536 1280; do
  if [ $g = 0 ]; then E=""; else E="PSIM_PTL_GRID=$g"; fi
  env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --steps 20 --warmup 5 > $O/b_${g}_$rep.json 2> $O/b_${g}_$rep.err || { echo FAIL $g; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${g}_$rep.json')); print('grid $g', $rep, 'ms/step %.3f node-round %.3f' % (d['ms_per_step'], d['roofline']['avg_launch_ms']))"
done; done
