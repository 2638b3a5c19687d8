"""Reads tools/cu_map.py's npz: per step, the CU / SIMD load of K1 (wave-busy cycles per SIMD,
summed over its waves), how much the CU end times spread, and whether a placement that balanced the
groups' measured costs over the CUs could shorten the step (the slowest CU's load vs the mean)."""
import sys

import numpy as np

z = np.load(sys.argv[1])
start, end, cu, simd, role, grp, xcc = (z[k] for k in ("start", "end", "cu", "simd", "role", "grp", "xcc"))
gscn, names = z["gscn"], z["names"]
K = start.shape[0]
for k in range(K):
    t0 = np.array([start[k][xcc[k] == x].min() if (xcc[k] == x).any() else 0 for x in range(16)])
    s, e = start[k] - t0[xcc[k]], end[k] - t0[xcc[k]]
    dur = e - s
    cus = np.unique(cu[k])
    cu_end = np.array([e[cu[k] == c].max() for c in cus])
    cu_busy = np.array([dur[cu[k] == c].sum() for c in cus])
    sim_busy = np.array([dur[(cu[k] == c) & (simd[k] == d)].sum() for c in cus for d in range(4)])
    if k in (0, 1, K - 1):
        print(f"step {k}: CUs {len(cus)} end med {np.median(cu_end):.0f} p90 {np.percentile(cu_end, 90):.0f} "
              f"max {cu_end.max():.0f}; CU wave-cycles mean {cu_busy.mean():.0f} max {cu_busy.max():.0f}; "
              f"SIMD wave-cycles mean {sim_busy.mean():.0f} max {sim_busy.max():.0f}")
# per-scenario group cost (sum of its four waves' durations, median over groups / steps)
gcost = {}
for k in range(K):
    t0 = np.array([start[k][xcc[k] == x].min() if (xcc[k] == x).any() else 0 for x in range(16)])
    dur = (end[k] - start[k])
    g = grp[k]
    for gi in np.unique(g):
        sc = gscn[gi]
        gcost.setdefault(sc, []).append(dur[g == gi].max())
for sc, v in sorted(gcost.items()):
    print(f"  {names[sc]:14s} groups x steps {len(v):5d}  longest wave median {np.median(v):.0f} p90 {np.percentile(v, 90):.0f}")
b0 = cu[0].reshape(-1, 4)[:, 0]
for k in range(1, K):
    bk = cu[k].reshape(-1, 4)[:, 0]
    print(f"step {k}: blocks on the same CU as step 0: {(bk == b0).mean():.2f}; same XCD: {((bk >> 8) == (b0 >> 8)).mean():.2f}")
