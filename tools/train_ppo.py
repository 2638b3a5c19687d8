#!/usr/bin/env python3
"""PPO training end-to-end on one MI355X (GPU box): the HIP env batch + drone2d_amd.ppo.

    python tools/train_ppo.py [--envs 65536] [--updates 30] [--scenario corridor | --curriculum]

One JSON line per update (timesteps, mean finished-episode return, losses, env-steps/s including
the policy forward passes and the PPO update) into gpurun_out/ppo.jsonl and on stdout.
``--curriculum`` trains as the reference does (mode='train': a fresh curriculum scenario per
reset, stage by the global step count, drone_2d_env.py:76-86 / 324-372), with the pool refreshed
(and the stage advanced) every ``--refresh`` updates.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--updates", type=int, default=30)
    ap.add_argument("--n-steps", type=int, default=16)
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--scenario", default="corridor")
    ap.add_argument("--curriculum", action="store_true")
    ap.add_argument("--pool", type=int, default=4096, help="curriculum pool size; 0: the fresh curriculum")
    ap.add_argument("--refresh", type=int, default=100, help="updates between curriculum pool refreshes")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-graph", action="store_true", help="eager minibatch updates (A/B against the HIP graph)")
    ap.add_argument("--autograd", action="store_true", help="autograd + torch Adam update (A/B against ManualStep)")
    a = ap.parse_args()

    import torch

    import drone2d_amd as d2
    from drone2d_amd.config import ENV_TRAIN_CONFIG
    from drone2d_amd.ppo import PPO, PPOConfig

    torch.cuda.set_device(0)
    kw = dict(ENV_TRAIN_CONFIG, scenario=a.scenario)
    if a.curriculum:
        kw.update(mode="curriculum", scenario="curriculum", sim_num=0, curriculum_seed=a.seed)
        if a.pool > 0:  # a host-generated pool; --pool 0: every reset on a fresh device-generated scenario
            kw["curriculum_pool"] = a.pool
    venv = d2.Drone2dVecEnv(a.envs, seed=a.seed, **kw)
    cfg = PPOConfig.gpu_defaults(n_steps=a.n_steps, batch_size=a.batch, n_epochs=a.epochs)
    cfg.graph = not a.no_graph
    cfg.manual = not a.autograd
    algo = PPO(venv, cfg, seed=a.seed)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    tag = ("_eager" if a.no_graph else "") + ("_autograd" if a.autograd else "")
    out = open(os.path.join(REPO, "gpurun_out", f"ppo{tag}.jsonl"), "w")
    t0 = time.perf_counter()
    for u in range(a.updates):
        if a.curriculum and a.pool > 0 and u and u % a.refresh == 0:
            # the reference's stage clock is the global step count (checkpoint names, :76-86)
            venv.refresh_curriculum(sim_num=algo.num_timesteps)
        rec = algo.learn(algo.num_timesteps + a.n_steps * a.envs)[-1]
        rec.update(update=u, wall_s=time.perf_counter() - t0)
        line = json.dumps({k: (round(v, 6) if isinstance(v, float) else v) for k, v in rec.items()})
        print(line, flush=True)
        out.write(line + "\n")
    total = algo.num_timesteps / (time.perf_counter() - t0)
    print(json.dumps({"envs": a.envs, "updates": a.updates, "timesteps": algo.num_timesteps, "graph": algo.use_graph, "manual": cfg.manual,
                      "env_steps_per_s_incl_learning": total}), flush=True)
    venv.close()


if __name__ == "__main__":
    main()
