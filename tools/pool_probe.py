"""Diagnostic (not product): curriculum-pool batch cost per step at 65 536 envs with the field-major
and the record-major build (argv: pool size, steps)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import drone2d_amd as d2  # noqa: E402
from drone2d_amd import _native  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402

pool = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
n = 65536
for lib in (_native.LIB_PATH,):
    venv = d2.Drone2dVecEnv(n, seed=0, with_info=False, native_lib=lib,
                            **dict(ENV_TRAIN_CONFIG, mode="curriculum", scenario="stage_3", curriculum_pool=pool))
    venv.reset(seed=0)
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = [torch.rand(n, 2, device="cuda", generator=g) * 2 - 1 for _ in range(16)]
    for k in range(100):
        venv.step(acts[k % 16])
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for k in range(steps):
        venv.step(acts[k % 16])
    b.record()
    torch.cuda.synchronize()
    print(f"pool {pool}, {os.path.basename(lib)}: {a.elapsed_time(b) * 1000 / steps:.1f} us per step", flush=True)
    venv.close()
