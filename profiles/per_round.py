"""Per-round durations of the node-round kernels over the last STEPS rounds
before the last TAIL (the bench's overlay drain: overlay.rounds_drained).
Usage: python profiles/per_round.py run_kernel_trace.csv [STEPS] [--tail TAIL]"""
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
out=[];cur=None
for r in rows:
    n=r['Kernel_Name']; d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000
    if 'k_relay' in n: cur={'relay':d}; out.append(cur)
    elif cur is not None:
        for k,tag in (('shuf','k_shuf'),('lite','k_consume_lite'),('lite','k_term'),('ptl','k_ptl('),('merge','k_merge'),('cons','k_consume('),('pt','k_pt(')):
            if tag in n: cur[k]=d
tail=int(sys.argv[sys.argv.index('--tail')+1]) if '--tail' in sys.argv else 0
if tail: out=out[:-tail]
steps=int(sys.argv[2]) if len(sys.argv)>2 and not sys.argv[2].startswith('--') else 20
last=out[-steps:]
for i,c in enumerate(last):
    print(i, ' '.join(f"{k}={v:7.1f}" for k,v in c.items()), f"sum={sum(c.values()):7.1f}")
tot={}
for c in last:
    for k,v in c.items(): tot[k]=tot.get(k,0)+v/len(last)
print('avg', ' '.join(f"{k}={v:7.1f}" for k,v in tot.items()), f"sum={sum(tot.values()):7.1f}")
