"""Diagnostic (not product): SIMD placement and per-role timelines of the step kernel when it
follows another step kernel vs when it follows the cache-fill kernel (tools/stamps.py build first).
Prints, per launch, how many CUs host two workgroups whose path waves (role 2) share a SIMD, and the
median / max wave end times per role."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import drone2d_amd as d2  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402

LIB = os.path.join(REPO, "tools", "_abl", "libd2d_stamps.so")
n = 65536
venv = d2.Drone2dVecEnv(n, seed=3, with_info=False, native_lib=LIB, **dict(ENV_TRAIN_CONFIG, scenario="corridor"))
lib = venv._lib
lib.d2d_debug_stamps.argtypes = [C.c_void_p, C.c_void_p]
nw = n // 64 * 4
venv.reset()
acts = [torch.rand(n, 2, device=venv.device) * 2 - 1 for _ in range(8)]
for k in range(40):  # the library launches the fill after every 16th step call
    venv.step(acts[k % 8])
res = {}
for call in range(41, 52):
    buf = torch.zeros(65536 + nw * 8, dtype=torch.int64, device=venv.device)
    lib.d2d_debug_stamps(venv._h, C.c_void_p(buf.data_ptr()))
    venv.step(acts[call % 8])
    torch.cuda.synchronize()
    s = buf[:nw * 8].cpu().numpy().reshape(-1, 4, 8)
    after = "fill" if call == 49 else ("fill2" if call == 50 else "step")
    hw = s[:, :, 7]
    cu = ((hw >> 32) << 16) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
    simd = (hw >> 4) & 3
    # per CU: SIMDs of the workgroups' path waves (role 2)
    per = {}
    for b in range(s.shape[0]):
        per.setdefault(int(cu[b, 2]), []).append(int(simd[b, 2]))
    clash = sum(1 for v in per.values() if len(set(v)) < len(v))
    wgs = [len(v) for v in per.values()]
    t0 = s[:, :, 0].min()
    end = (s[:, :, 6] - t0)
    line = (f"call {call} ({after:5s}) CUs {len(per)} wg/CU {min(wgs)}-{max(wgs)} CUs-with-W2-clash {clash:3d} "
            f"end median {np.median(end):8.0f} max {end.max():8.0f} by role max " +
            " ".join(f"{end[:, r].max():7.0f}" for r in range(4)))
    print(line, flush=True)
venv.close()
