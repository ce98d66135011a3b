import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
out=[];cur=None
for r in rows:
    n=r['Kernel_Name']; d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000
    if 'k_relay' in n: cur={'relay':d}; out.append(cur)
    elif cur is not None:
        for k,tag in (('shuf','k_shuf'),('lite','k_consume_lite'),('ptl','k_ptl('),('merge','k_merge'),('cons','k_consume('),('pt','k_pt(')):
            if tag in n: cur[k]=d
last=out[-int(sys.argv[2]) if len(sys.argv)>2 else -20:]
for i,c in enumerate(last):
    print(i, ' '.join(f"{k}={v:7.1f}" for k,v in c.items()), f"sum={sum(c.values()):7.1f}")
tot={}
for c in last:
    for k,v in c.items(): tot[k]=tot.get(k,0)+v/len(last)
print('avg', ' '.join(f"{k}={v:7.1f}" for k,v in tot.items()), f"sum={sum(tot.values()):7.1f}")
