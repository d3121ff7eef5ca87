"""Per-level breakdown of a KZG get_proof kernel trace (rocprofv3 --kernel-trace CSV of tools/kzg_getproof.py).
usage: python tools/getproof_levels.py <run_kernel_trace.csv>"""
import csv, sys
from collections import defaultdict
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
starts=[i for i,r in enumerate(rows) if 'k_sub_const' in r['Kernel_Name']]
i0=starts[-1]
tops=[j for j in range(i0,len(rows)) if 'k_top_diff' in rows[j]['Kernel_Name']][:24]
tot_w=0
for li,(a,b) in enumerate(zip(tops, tops[1:]+[None])):
    if b is None: break
    agg=defaultdict(float); cnt=defaultdict(int)
    for r in rows[a:b]:
        n=r['Kernel_Name'].split('(')[0].replace('void ','').replace('zk::','')[:18]
        agg[n]+= (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3; cnt[n]+=1
    wall=(int(rows[b]['Start_Timestamp'])-int(rows[a]['Start_Timestamp']))/1e3
    tot_w+=wall
    busy=sum(agg.values())
    top=sorted(agg.items(), key=lambda x:-x[1])[:5]
    print(f'L{li:2d} 2^{23-li:2d}: wall {wall:6.0f} busy {busy:6.0f} n_k {sum(cnt.values()):3d} |', ', '.join(f'{k}:{v:.0f}x{cnt[k]}' for k,v in top))
# the rest of the call: the last level and, with level batching, the one MSM
# pass over the batched quotients — up to the next call's first kernel (a
# commit starts with k_convert, a get_proof with k_sub_const)
last = tops[-1]
lf = [j for j in range(i0, len(rows)) if 'k_fold<' in rows[j]['Kernel_Name']][len(tops) - 1]  # the last level's fold
end = next((j for j in range(lf + 1, len(rows)) if 'k_convert' in rows[j]['Kernel_Name']
            or 'k_sub_const' in rows[j]['Kernel_Name']), len(rows))
agg = defaultdict(float)
cnt = defaultdict(int)
for r in rows[last:end]:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('zk::', '')[:18]
    agg[n] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    cnt[n] += 1
wall = (int(rows[end - 1]['End_Timestamp']) - int(rows[last]['Start_Timestamp'])) / 1e3
tot_w += wall
top = sorted(agg.items(), key=lambda x: -x[1])[:6]
print(f'last level + batched pass: wall {wall:6.0f} busy {sum(agg.values()):6.0f} |',
      ', '.join(f'{k}:{v:.0f}x{cnt[k]}' for k, v in top))
print('sum of levels', tot_w/1e3, 'ms')
