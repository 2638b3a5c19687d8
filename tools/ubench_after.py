"""Diagnostic (not product): does a kernel launched between two d2d_step launches slow the next
step kernel down?  Eager loop at 65 536 corridor envs; between some steps a torch fill kernel of a
chosen size runs.  Run under rocprofv3 --kernel-trace and read the step kernel's duration by its
predecessor (tools/ubench_after_report.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import drone2d_amd as d2  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402

venv = d2.Drone2dVecEnv(65536, seed=1, **dict(ENV_TRAIN_CONFIG, scenario="corridor"))
venv.reset()
dev = venv.device
acts = [(torch.rand(65536, 2, device=dev) * 2 - 1) for _ in range(8)]
buf = torch.zeros(1 << 24, device=dev)
for k in range(40):
    venv.step(acts[k % 8])
torch.cuda.synchronize()
# elements per dummy fill: ~ numel / (256 threads x 4 per thread) workgroups
for n_el in (2048, 262144, 1048576, 4194304, 16777216):
    for rep in range(6):
        venv.step(acts[rep % 8])
        buf[:n_el].fill_(float(rep))
        venv.step(acts[(rep + 1) % 8])
        venv.step(acts[(rep + 2) % 8])
    torch.cuda.synchronize()
print("done")
