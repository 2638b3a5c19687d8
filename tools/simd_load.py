"""Diagnostic (not product): where the time of one step goes, per CU and SIMD, from the stamps build
(tools/stamps.py build).  For one step after a warmup: per wave its role, group (scenario), SIMD and
start / end (s_memtime, per-XCD clock: times relative to the earliest start on the same XCD);
prints the distribution of CU end times and, for the slowest CUs, each SIMD's waves."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import drone2d_amd as d2  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scenario", default="corridor")
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--warm", type=int, default=300)
ap.add_argument("--dump", default="")
a = ap.parse_args()
MIXED = ["perpendicular", "parallel", "S_parallel", "corridor", "S_corridor", "large", "impossible"]
scn = MIXED if a.scenario == "mixed" else a.scenario
LIB = os.path.join(REPO, "tools", "_abl", "libd2d_stamps.so")
n = a.envs
venv = d2.Drone2dVecEnv(n, seed=3, with_info=False, native_lib=LIB, **dict(ENV_TRAIN_CONFIG, scenario=scn))
lib = venv._lib
lib.d2d_debug_stamps.argtypes = [C.c_void_p, C.c_void_p]
nw = (n + 63) // 64 * 4
venv.reset()
for k in range(a.warm):
    venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
buf = torch.zeros(65536 + nw * 8 + 4096, dtype=torch.int64, device=venv.device)
lib.d2d_debug_stamps(venv._h, C.c_void_p(buf.data_ptr()))
venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
torch.cuda.synchronize()
s = buf[:nw * 8].cpu().numpy().reshape(-1, 8).astype(np.int64)
hw = s[:, 7]
xcc = (hw >> 32) & 0xF
role = (hw >> 36) & 3
grp = (hw >> 40) - 1
cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
simd = (hw >> 4) & 3
es = venv.env_scenario
slot_env = None
lay = venv.group_layout()
gscn = lay[1] if lay is not None else np.zeros(nw // 4, np.int32)
names = [x.name for x in venv.scenarios]
t0 = np.zeros(16, np.int64)
for x in range(16):
    m = xcc == x
    if m.any():
        t0[x] = s[m, 0].min()
start = s[:, 0] - t0[xcc]
end = s[:, 6] - t0[xcc]
cus = {}
for w in range(len(s)):
    cus.setdefault(int(cu[w]), []).append(w)
cu_end = {c: end[ws].max() for c, ws in cus.items()}
v = np.array(sorted(cu_end.values()))
print(f"{a.scenario}: waves {len(s)}, CUs {len(cus)}; CU end cycles: median {np.median(v):.0f} p90 {np.percentile(v, 90):.0f} "
      f"max {v.max():.0f}; wave end by role median " + " ".join(f"{np.median(end[role == r]):.0f}" for r in range(4)))
for c in sorted(cu_end, key=cu_end.get)[-3:] + sorted(cu_end, key=cu_end.get)[:1]:
    print(f"  CU {c:5d} end {cu_end[c]:.0f}")
    for sd in range(4):
        ws = [w for w in cus[c] if simd[w] == sd]
        desc = ", ".join(f"r{role[w]}:{names[gscn[grp[w]]] if grp[w] >= 0 and gscn[grp[w]] >= 0 else '?'}"
                         f"[{start[w]:.0f}-{end[w]:.0f}]" for w in ws)
        print(f"     simd {sd}: {desc}")
if a.dump:
    np.savez(a.dump, block=np.arange(len(s)) // 4, wave=np.arange(len(s)) % 4, cu=cu, simd=simd, role=role, grp=grp,
             start=start, end=end, gscn=gscn)
venv.close()
