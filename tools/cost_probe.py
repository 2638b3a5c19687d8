"""Diagnostic (not product): the mixed batch (65 536 envs, env i on scenario i mod 7) stepped with
two scenario-cost tables for the co-residency balance (d2d_set_scenario_costs; placement only, the
results are the same bit for bit): the table in config.py and the one passed as JSON, alternating,
ms per step over the eager loop.

    python tools/cost_probe.py '{"perpendicular": 26.4, ...}' [rounds]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import drone2d_amd as d2  # noqa: E402
from drone2d_amd import config, env  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402
from bench import MIXED  # noqa: E402

new = json.loads(sys.argv[1])
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
old = dict(config.SCENARIO_STEP_COST)
n = 65536
res = {"config.py": [], "probe": []}
for r in range(rounds):
    for tag, table in (("config.py", old), ("probe", new)):
        env.SCENARIO_STEP_COST.clear()
        env.SCENARIO_STEP_COST.update(table)
        venv = d2.Drone2dVecEnv(n, seed=1, with_info=False, env_scenario=np.arange(n) % 7,
                                **dict(ENV_TRAIN_CONFIG, scenario=MIXED))
        venv.reset()
        acts = [torch.rand(n, 2, device=venv.device) * 2 - 1 for _ in range(8)]
        for k in range(300):
            venv.step(acts[k % 8])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(1000):
            venv.step(acts[k % 8])
        e1.record()
        torch.cuda.synchronize()
        res[tag].append(e0.elapsed_time(e1))  # ms per 1000 steps = us per step
        venv.close()
print(json.dumps({k: [round(x, 2) for x in v] for k, v in res.items()}))
