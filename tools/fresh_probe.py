"""Diagnostic (not product): the fresh curriculum's cost per step at 65 536 envs -- steps a
fresh-curriculum batch (mode='curriculum', every reset on its own device-generated scenario) with
random actions and prints ms per step (HIP events) for the eager loop; run under rocprofv3
--kernel-trace --stats for the per-kernel split (d2d_fresh_kernel = K5)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import drone2d_amd as d2  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 400
lib = sys.argv[3] if len(sys.argv) > 3 else None  # an alternative build (tools/variants.py)
venv = d2.Drone2dVecEnv(n, seed=0, with_info=False, native_lib=lib,
                        **dict(ENV_TRAIN_CONFIG, mode="curriculum", scenario="curriculum", sim_num=0))
venv.reset(seed=0)
g = torch.Generator(device="cuda").manual_seed(0)
acts = [torch.rand(n, 2, device="cuda", generator=g) * 2 - 1 for _ in range(16)]
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for k in range(100):
    venv.step(acts[k % 16])
torch.cuda.synchronize()
a.record()
for k in range(steps):
    venv.step(acts[k % 16])
b.record()
torch.cuda.synchronize()
print(f"fresh curriculum{' (' + os.path.basename(lib) + ')' if lib else ''}, {n} envs: {a.elapsed_time(b) * 1000 / steps:.1f} us per step "
      f"({n * steps / (a.elapsed_time(b) / 1000) / 1e9:.3f} G env-steps/s, eager)", flush=True)
