#!/bin/bash
# PMC traffic records (per kernel) of the B, D and E-at-2^26 lines, then the
# lines themselves reading them back.  Usage (GPU box, repo root): bash profiles/r04/pmc_lines.sh TAG
TAG=${1:-pl}
O=gpurun_out/$TAG
mkdir -p $O
E26S="--workload E --schedule survey --nodes 67108864 --steps 140 --warmup 5"
bash profiles/run_pmc.sh ${TAG}_B --workload B --steps 20 --warmup 5 | tail -1 || exit 1
bash profiles/run_pmc.sh ${TAG}_D --workload D --steps 20 --warmup 5 | tail -1 || exit 1
bash profiles/run_pmc.sh ${TAG}_E26s $E26S --no-check | tail -1 || exit 1
for n in B D; do timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $n --steps 20 --warmup 5 > $O/bench_$n.json 2> $O/$n.err || exit 1; done
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-check $E26S > $O/bench_E26s.json 2> $O/E26s.err || exit 1
for f in $O/bench_*.json; do python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[1].split('/')[-1], '%.3g' % d['value'], 'ms/step %.3f frac %.4f traffic %s alg %.4g' % (d['ms_per_step'], r['frac'], r.get('traffic'), r['alg_bytes_per_launch']))" $f; done
