#!/usr/bin/env python3
"""Timeline of the last prove in a rocprofv3 --kernel-trace csv (tools/prove_only.py or bench.py):
every dispatch of the step (start, duration, kernel, grid, queue = stream), the union of busy
intervals and the largest idle gaps.  A step starts at the side stream's first transform.

usage: step_timeline.py run_kernel_trace.csv [all]
"""
import csv,re,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
def nm(r):
    n=r['Kernel_Name']; n=re.sub(r'\(.*','',n); n=n.replace('void ','').replace('sg::','')
    return n[:34]+f" g={r['Grid_Size_X']}x{r['Grid_Size_Y']} q{r['Queue_Id']}"
side=[i for i,r in enumerate(rows) if r['Queue_Id']!='1' and 'k_ntt_first' in r['Kernel_Name']]
gmax=max((int(rows[i]['Grid_Size_X']) for i in side), default=0)
starts=[i for i in side if int(rows[i]['Grid_Size_X'])==gmax]
# step start = side-stream randomizer LDE; keep those followed by gather_stride soon
print('candidate starts', len(starts))
step_starts=starts[-3:]
last=step_starts[-1]
end=len(rows)
# end of step: before next big gap > 2ms
t_prev=int(rows[last]['End_Timestamp'])
for j in range(last, len(rows)):
    s=int(rows[j]['Start_Timestamp'])
    if s - t_prev > 2e6: end=j; break
    t_prev=max(t_prev,int(rows[j]['End_Timestamp']))
seg=rows[last:end]
t0=int(seg[0]['Start_Timestamp'])
T=max(int(r['End_Timestamp']) for r in seg)-t0
iv=sorted((int(r['Start_Timestamp'])-t0,int(r['End_Timestamp'])-t0,nm(r)) for r in seg)
busy=0; cur_s,cur_e=iv[0][0],iv[0][1]; gaps=[]
prevname=iv[0][2]
for s,e,n in iv[1:]:
    if s>cur_e:
        busy+=cur_e-cur_s; gaps.append((s-cur_e,cur_e,prevname,n)); cur_s,cur_e=s,e
    else: cur_e=max(cur_e,e)
    if e>=cur_e: prevname=n
busy+=cur_e-cur_s
print(f"step {len(seg)} kernels span {T/1e3:.1f} us busy {busy/1e3:.1f} us idle {(T-busy)/1e3:.1f} us")
gaps.sort(reverse=True)
for g,at,a,b in gaps[:40]:
    print(f"gap {g/1e3:7.1f} us at {at/1e3:8.1f}  after {a}  before {b}")
if len(sys.argv)>2:
    for s,e,n in iv: print(f"{s/1e3:9.1f} {(e-s)/1e3:8.1f} {n}")
