"""Diagnostic (not product): is the dispatcher's workgroup -> CU placement of K1 stable from step to
step when the step loop replays as a graph (back-to-back launches)?  Captures 16 steps with the
stamps build (tools/stamps.py build), each step stamping into its own buffer, replays once and saves
per step and wave: CU id, SIMD, role, group, start / end (s_memtime) into an npz."""
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
ap.add_argument("--scenario", default="mixed")
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--warm", type=int, default=300)
ap.add_argument("--out", required=True)
a = ap.parse_args()
MIXED = ["perpendicular", "parallel", "S_parallel", "corridor", "S_corridor", "large", "impossible"]
scn = MIXED if a.scenario == "mixed" else a.scenario
LIB = os.path.join(REPO, "tools", "_abl", "libd2d_stamps.so")
n = a.envs
venv = d2.Drone2dVecEnv(n, seed=3, with_info=False, native_lib=LIB, **dict(ENV_TRAIN_CONFIG, scenario=scn))
lib = venv._lib
lib.d2d_debug_stamps.argtypes = [C.c_void_p, C.c_void_p]
nw = (n + 63) // 64 * 4
K = 16
bufs = [torch.zeros(65536 + nw * 8 + 4096, dtype=torch.int64, device=venv.device) for _ in range(K)]
acts = torch.rand(K, n, 2, device=venv.device) * 2 - 1
venv.reset()
for k in range(a.warm):
    venv.step(acts[k % K])
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for k in range(K):
        lib.d2d_debug_stamps(venv._h, C.c_void_p(bufs[k].data_ptr()))
        venv.step(acts[k])
for _ in range(4):
    g.replay()
torch.cuda.synchronize()
S = np.stack([b[:nw * 8].cpu().numpy().reshape(-1, 8) for b in bufs])  # [K, waves, 8]
hw = S[..., 7]
xcc = (hw >> 32) & 0xF
cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
lay = venv.group_layout()
gs = lay[1] if lay is not None else np.zeros((n + 63) // 64, np.int32)
np.savez(a.out, start=S[..., 0], end=S[..., 6], cu=cu, simd=(hw >> 4) & 3, role=(hw >> 36) & 3,
         grp=(hw >> 40) - 1, xcc=xcc, gscn=gs, names=np.array([s.name for s in venv.scenarios]))
same = [(cu[k].reshape(-1, 4)[:, 0] == cu[0].reshape(-1, 4)[:, 0]).mean() for k in range(K)]
print(a.scenario, "block->CU same as step 0:", " ".join(f"{x:.2f}" for x in same))
venv.close()
