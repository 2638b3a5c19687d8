"""Diagnostic (not product): K5 (d2d_fresh_gen_kernel) duration against the number of scenarios it
generates in one launch -- the reset (n items), per-step launches (~n/76 items), and a recipe restore
(2n items).  Run under ``rocprofv3 --kernel-trace`` and read the gen-kernel rows in launch order."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import drone2d_amd as d2  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
venv = d2.Drone2dVecEnv(n, seed=0, with_info=False,
                        **dict(ENV_TRAIN_CONFIG, mode="curriculum", scenario="curriculum", sim_num=3_000_000))
venv.reset(seed=0)
torch.cuda.synchronize()
for k in range(40):
    venv.step(torch.rand(n, 2, device="cuda") * 2 - 1)
torch.cuda.synchronize()
keys, clocks, clock = venv.fresh_recipes()
print("valid slots", int((keys >= 0).sum()), "of", len(keys), flush=True)
for rep in range(3):
    sd = venv.state_dict()
    venv.load_state_dict(sd)   # regenerates every valid slot from its recipe (one K5 launch)
    torch.cuda.synchronize()
print("done", flush=True)
