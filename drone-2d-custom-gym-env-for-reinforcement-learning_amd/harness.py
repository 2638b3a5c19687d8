"""Test harness on the batched env: the reference's ``mode == "test"`` loop
(main.py:242-327) -- run a policy until every env finishes its first episode, then report the same
metrics and files (``results.txt`` lines, ``apes/collisions/rewards/time_spent.npy``) -- with all
envs of a scenario stepping in one batch instead of 100 sequential runs.

``MlpActor`` is SB3's default ``MlpPolicy`` actor (27-64-64-2, tanh; policy_kwargs {} in the
shipped agents), loaded from the float32 weights extracted from an agent zip
(tests/golden/make_agent_fixture.py).  ``model.predict(obs)`` in the reference is stochastic
(deterministic=False): a = clip(mean + exp(log_std) * N(0, 1), -1, 1).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from . import abi
from .env import info_dicts


class MlpActor(torch.nn.Module):
    def __init__(self, w: dict):
        super().__init__()
        t = {k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in w.items()}
        self.l0 = torch.nn.Linear(27, 64)
        self.l1 = torch.nn.Linear(64, 64)
        self.out = torch.nn.Linear(64, 2)
        with torch.no_grad():
            self.l0.weight.copy_(t["mlp_extractor_policy_net_0_weight"])
            self.l0.bias.copy_(t["mlp_extractor_policy_net_0_bias"])
            self.l1.weight.copy_(t["mlp_extractor_policy_net_2_weight"])
            self.l1.bias.copy_(t["mlp_extractor_policy_net_2_bias"])
            self.out.weight.copy_(t["action_net_weight"])
            self.out.bias.copy_(t["action_net_bias"])
        self.register_buffer("log_std", t["log_std"].clone())

    @classmethod
    def from_npz(cls, path: str) -> "MlpActor":
        with np.load(path, allow_pickle=False) as z:
            return cls({k: z[k] for k in z.files})

    def forward(self, obs: torch.Tensor) -> torch.Tensor:
        return self.out(torch.tanh(self.l1(torch.tanh(self.l0(obs)))))

    @torch.no_grad()
    def act(self, obs: torch.Tensor, deterministic: bool = False, generator: torch.Generator | None = None):
        mean = self(obs)
        if not deterministic:
            noise = torch.randn(mean.shape, device=mean.device, dtype=mean.dtype, generator=generator)
            mean = mean + torch.exp(self.log_std) * noise
        return torch.clamp(mean, -1.0, 1.0)


def run_first_episodes(venv, policy: MlpActor, *, deterministic: bool = False, seed: int = 0,
                       max_steps: int | None = None, n_obstacles: int | None = None,
                       flight_paths: bool = False) -> dict:
    """Step ``venv`` (with info rows) under ``policy`` until every env has finished its first
    episode; per-episode records as the reference's test loop keeps them (main.py:273-281).

    ``flight_paths``: also return ``flight_xy`` [steps, episodes, 2] (NaN past each episode's
    end; ``flight_path_lists`` turns it into the JSON value), each episode's
    ``info['flight_path']`` -- the frame position
    after every step as (x, screen_height - y), one entry per env step including the last
    (drone_2d_env.py:409-415, 984-986; saved as JSON by main.py:307-308).  The positions are decoded
    from the observation (obs[6:8] = 2p/(W,H) - 1, the terminal observation on the last step), so
    they carry the float32 observation's rounding (<= 1e-4 px at 1300 px) where the reference
    records the fp64 body position; the buffer stays on the device (8 B per env-step) until the
    episodes are done."""
    dev = venv.device
    gen = torch.Generator(device=dev).manual_seed(seed)
    policy = policy.to(dev)
    obs = venv.reset(seed=seed)
    n = venv.num_envs
    finished = torch.zeros(n, dtype=torch.bool, device=dev)
    rows = torch.zeros(n, abi.INFO_DIM, dtype=torch.float32, device=dev)
    cap = max_steps if max_steps is not None else int(venv.kwargs["n_steps"]) + 1
    nobs = n_obstacles if n_obstacles is not None else len(venv.scenarios[0].circles)
    pos = torch.empty(cap, n, 2, dtype=torch.float32, device=dev) if flight_paths else None
    steps = 0
    for t in range(cap):
        a = policy.act(obs, deterministic=deterministic, generator=gen)
        obs, rew, term, trunc, info = venv.step(a)
        done = term | trunc
        new = done & ~finished
        rows[new] = info[new]
        if pos is not None:
            pos[t] = torch.where(done[:, None], venv.terminal_obs[:, 6:8].to(dev), obs[:, 6:8])
        steps = t + 1
        finished |= done
        if bool(finished.all()):
            break
    idx = torch.nonzero(finished).flatten()
    rows = rows[idx].cpu().numpy()
    recs = [info_dicts(r, nobs) for r in rows]
    out = {
        "successes": int(sum(d["n_successful_runs"] == 1 for d in recs)),
        "fails": int(sum(d["n_failed_runs"] == 1 for d in recs)),
        "collisions": np.array([d["n_collisions"] for d in recs], np.int64),
        "apes": np.array([d["APE"] for d in recs], np.float64),
        "time_spent": np.array([d["env_steps"] for d in recs], np.int64),
        "rewards": np.array([d["total_reward"] for d in recs], np.float64),
        "unfinished": int(n - len(recs)),
    }
    if pos is not None:
        w, h = float(venv.kwargs["screensize_x"]), float(venv.kwargs["screensize_y"])
        xy = pos[:steps, idx].double().cpu().numpy()  # [steps, finished envs, 2]
        fl = np.stack([(xy[..., 0] + 1.0) * w / 2.0, h - (xy[..., 1] + 1.0) * h / 2.0], -1)
        fl[np.arange(steps)[:, None] >= out["time_spent"][None, :]] = np.nan  # after each episode's end
        out["flight_xy"] = fl
    return out


def flight_path_lists(m: dict) -> list:
    """``m["flight_xy"]`` as the reference's ``flight_paths`` JSON value: one list of [x, y] per
    episode, ``env_steps`` entries long (main.py:278, 307-308)."""
    fl = m["flight_xy"]
    return [fl[:T, j].tolist() for j, T in enumerate(m["time_spent"])]


def summary(m: dict) -> dict:
    """The numbers of the reference's results.txt (main.py:318-325)."""
    runs = m["successes"] + m["fails"]
    col = int(m["collisions"].sum())
    return {"Successes": m["successes"], "Fails": m["fails"], "Collisions": col,
            "Success rate": m["successes"] / max(runs, 1), "Collision rate": col / max(runs, 1),
            "Average APE": float(np.mean(m["apes"])) if len(m["apes"]) else float("nan"),
            "Average flight time": float(np.mean(m["time_spent"])) if len(m["time_spent"]) else float("nan")}


def write_results(m: dict, out_dir: str, scenario: str, agent_nr: str, agent_path: str):
    """The reference's per-scenario files: results.txt + collisions/rewards/apes/time_spent .npy
    (+ the ``flight_paths`` JSON when ``m`` carries them), main.py:307-326."""
    os.makedirs(out_dir, exist_ok=True)
    for k in ("collisions", "rewards", "apes", "time_spent"):
        np.save(os.path.join(out_dir, f"{k}.npy"), m[k])
    if "flight_xy" in m:
        with open(os.path.join(out_dir, "flight_paths"), "w") as f:
            json.dump(flight_path_lists(m), f)
    s = summary(m)
    with open(os.path.join(out_dir, f"{scenario}_{agent_nr}_results.txt"), "w") as f:
        for k in ("Successes", "Fails", "Collisions", "Success rate", "Collision rate", "Average APE",
                  "Average flight time"):
            f.write(f"{k}: {s[k]}\n")
        f.write(f"Agent path: {agent_path}\n")
    return s


__all__ = ["MlpActor", "run_first_episodes", "flight_path_lists", "summary", "write_results"]
