"""Reads tools/cu_map.py's npz: per scenario, the duration of its workgroups (longest wave, s_memtime
cycles) split by how many other heavy groups (S_parallel, S_corridor, large, straddling) share the
CU, the CU spans and the slowest workgroup of every step (the step's length)."""
import numpy as np, sys
z=np.load(sys.argv[1])
names=list(z['names']); gscn=z['gscn']
heavyset={'S_parallel','S_corridor','large'}
res={}; spans=[]; wgmax=[]
for k in range(16):
    start,end,cu,grp=(z[x][k] for x in ("start","end","cu","grp"))
    mx=0
    for c in np.unique(cu):
        m=np.flatnonzero(cu==c); gs=np.unique(grp[m])
        sc=[gscn[g] for g in gs]
        heavy=[1 if (s<0 or names[s] in heavyset) else 0 for s in sc]
        spans.append(end[m].max()-start[m].min())
        for g,s,h in zip(gs,sc,heavy):
            mm=m[grp[m]==g]; d=end[mm].max()-start[mm].min(); mx=max(mx,d)
            nm='straddle' if s<0 else names[s]
            res.setdefault((nm,sum(heavy)-h),[]).append(d)
    wgmax.append(mx)
for key in sorted(res): v=res[key]; print('%-14s others-heavy=%d n=%5d med %6.0f p90 %6.0f max %6.0f'%(key[0],key[1],len(v),np.median(v),np.percentile(v,90),max(v)))
print('CU span med %.0f p90 %.0f max %.0f; per-step max WG: %s'%(np.median(spans),np.percentile(spans,90),max(spans), ' '.join('%.0f'%x for x in wgmax)))
