import csv, sys
import gzip
rows=list(csv.DictReader((gzip.open(sys.argv[1], 'rt') if sys.argv[1].endswith('.gz') else open(sys.argv[1]))))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
marker = sys.argv[2] if len(sys.argv) > 2 else 'k_gauss_bwd_live'  # (one launch per step)
gb=[i for i,r in enumerate(rows) if marker in r['Kernel_Name'] and 'k_gauss_bwd_live' not in r['Kernel_Name'].replace(marker, '', 1) or (marker == 'k_gauss_bwd_live' and 'k_gauss_bwd_live' in r['Kernel_Name'])]
a,b=gb[-6],gb[-5]
t0=int(rows[a]['Start_Timestamp'])
busy=[]
for r in rows[a:b+1]:
    s=(int(r['Start_Timestamp'])-t0)/1e3; e=(int(r['End_Timestamp'])-t0)/1e3
    busy.append((s,e))
    print(f"{s:8.1f} {e:8.1f} {e-s:6.1f} q{r['Queue_Id']:>2} s{r['Stream_Id']:>2} {r['Kernel_Name'][:60]}")
busy.sort(); cur=busy[0][1]; idle=0
for s,e in busy[1:]:
    if s>cur: idle+=s-cur
    cur=max(cur,e)
print("span",busy[-1][0],"idle",idle)
