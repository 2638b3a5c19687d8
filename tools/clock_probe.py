"""Diagnostic (not product): are the first steps after a reset slow because of the env state (all
episodes young) or because the GPU has just woken up?  Times 25 eager steps right after a reset,
(a) on a freshly started process and (b) after the GPU has been kept busy for ~0.3 s by another env
batch; prints per-step HIP-event times."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import drone2d_amd as d2  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402


def run(venv, n_steps, acts):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n_steps + 1)]
    torch.cuda.synchronize()
    ev[0].record()
    for k in range(n_steps):
        venv.step(acts[k % len(acts)])
        ev[k + 1].record()
    torch.cuda.synchronize()
    return [round(ev[k].elapsed_time(ev[k + 1]) * 1000, 1) for k in range(n_steps)]


n = 65536
kw = dict(ENV_TRAIN_CONFIG, scenario="corridor")
gen = torch.Generator(device="cuda").manual_seed(0)
acts = [torch.rand(n, 2, device="cuda", generator=gen) * 2 - 1 for _ in range(25)]
a = d2.Drone2dVecEnv(n, seed=0, with_info=False, **kw)
a.reset(seed=0)
print("cold, after reset:", run(a, 25, acts), flush=True)
b = d2.Drone2dVecEnv(n, seed=1, with_info=False, **kw)
b.reset(seed=1)
run(b, 300, acts)
a.reset(seed=0)
print("warm GPU, after reset:", run(a, 25, acts), flush=True)
print("warm GPU, steps 300+ of the other batch:", run(b, 25, acts), flush=True)
