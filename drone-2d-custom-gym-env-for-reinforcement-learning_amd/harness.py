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
    """SB3 MlpPolicy actor.  ``batch_invariant=True`` evaluates every linear layer as a fixed-order
    sum of element-wise products (bias + x_0 w_0 + x_1 w_1 + ...): each env's action is then a
    function of its own observation alone, bit for bit independent of the batch it sits in, so a
    run sharded over ranks reproduces one unsharded batch exactly (a GEMM may pick a different
    kernel -- and summation order -- for a different batch size)."""

    def __init__(self, w: dict, batch_invariant: bool = False):
        super().__init__()
        t = {k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in w.items()}
        self.l0 = torch.nn.Linear(27, 64)
        self.l1 = torch.nn.Linear(64, 64)
        self.out = torch.nn.Linear(64, 2)
        self.batch_invariant = batch_invariant
        with torch.no_grad():
            self.l0.weight.copy_(t["mlp_extractor_policy_net_0_weight"])
            self.l0.bias.copy_(t["mlp_extractor_policy_net_0_bias"])
            self.l1.weight.copy_(t["mlp_extractor_policy_net_2_weight"])
            self.l1.bias.copy_(t["mlp_extractor_policy_net_2_bias"])
            self.out.weight.copy_(t["action_net_weight"])
            self.out.bias.copy_(t["action_net_bias"])
        self.register_buffer("log_std", t["log_std"].clone())

    @classmethod
    def from_npz(cls, path: str, batch_invariant: bool = False) -> "MlpActor":
        with np.load(path, allow_pickle=False) as z:
            return cls({k: z[k] for k in z.files}, batch_invariant=batch_invariant)

    @staticmethod
    def _lin_fixed(x: torch.Tensor, lin: torch.nn.Linear) -> torch.Tensor:
        y = lin.bias.expand(x.shape[0], -1).clone()
        w = lin.weight.t()  # [in, out]
        for k in range(w.shape[0]):
            y = y + x[:, k:k + 1] * w[k]
        return y

    def forward(self, obs: torch.Tensor) -> torch.Tensor:
        if self.batch_invariant:
            h = torch.tanh(self._lin_fixed(obs, self.l0))
            h = torch.tanh(self._lin_fixed(h, self.l1))
            return self._lin_fixed(h, self.out)
        return self.out(torch.tanh(self.l1(torch.tanh(self.l0(obs)))))

    @torch.no_grad()
    def act(self, obs: torch.Tensor, deterministic: bool = False, generator: torch.Generator | None = None,
            noise: torch.Tensor | None = None):
        """a = clip(mean + exp(log_std) * N(0, 1), -1, 1); ``noise`` supplies the N(0, 1) draws
        (the harness passes each shard its block of one global draw)."""
        mean = self(obs)
        if not deterministic:
            if noise is None:
                noise = torch.randn(mean.shape, device=mean.device, dtype=mean.dtype, generator=generator)
            mean = mean + torch.exp(self.log_std) * noise
        return torch.clamp(mean, -1.0, 1.0)


def _dist_world():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist, dist.get_rank(), dist.get_world_size()
    return None, 0, 1


def run_first_episodes(venv, policy: MlpActor, *, deterministic: bool = False, seed: int = 0,
                       max_steps: int | None = None, n_obstacles: int | None = None,
                       flight_paths: bool = False, check_every: int = 16, gather: bool = True,
                       policy_device=None) -> dict:
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
    episodes are done.

    The loop never waits on the device per step: finished episodes' info rows are kept by a
    masked select on the device and the "all done" test reads back one flag every
    ``check_every`` steps.

    Sharded (torch.distributed initialised, world > 1, every rank passing its shard of one global
    batch: ``shard.make_shard_venv``): each rank steps its own envs; the policy noise of global env
    i at step t is entry i of one global N(0, 1) draw per step (the same generator on every rank),
    so the episodes are those of one unsharded batch; at the end rank 0 gathers every rank's
    records in global env order (``gather``) and the returned dict covers the whole batch (other
    ranks get their own shard's).  Use a ``batch_invariant`` policy for bit-identical actions.

    ``policy_device``: where the policy and its noise run (default: the env's device).  The
    parity tests pass "cpu" for the HIP batch and the CPU oracle alike, so both see the same
    actions for the same observations (a GPU tanh or N(0, 1) stream is not the CPU one)."""
    dev = venv.device
    pdev = torch.device(policy_device) if policy_device is not None else dev
    dist, rank, world = _dist_world()
    gen = torch.Generator(device=pdev).manual_seed(seed)
    policy = policy.to(pdev)
    obs = venv.reset(seed=seed)
    n = venv.num_envs
    offset = int(getattr(venv.cfg, "env_id_base", 0)) if world > 1 else 0
    n_total = n
    if world > 1:
        counts = [None] * world
        dist.all_gather_object(counts, n)
        n_total = int(sum(counts))
    finished = torch.zeros(n, dtype=torch.bool, device=dev)
    rows = torch.zeros(n, abi.INFO_DIM, dtype=torch.float32, device=dev)
    cap = max_steps if max_steps is not None else int(venv.kwargs["n_steps"]) + 1
    nobs = n_obstacles if n_obstacles is not None else len(venv.scenarios[0].circles)
    pos = torch.full((cap, n, 2), float("nan"), dtype=torch.float32, device=dev) if flight_paths else None
    for t in range(cap):
        noise = None
        if not deterministic:
            noise = torch.randn((n_total, 2), device=pdev, dtype=torch.float32, generator=gen)[offset:offset + n]
        a = policy.act(obs.to(pdev), deterministic=deterministic, noise=noise)
        obs, rew, term, trunc, info = venv.step(a)
        done = term | trunc
        new = done & ~finished
        rows = torch.where(new[:, None], info.to(dev), rows)
        if pos is not None:
            xy = torch.where(done[:, None], venv.terminal_obs[:, 6:8].to(dev), obs[:, 6:8])
            pos[t] = torch.where(finished[:, None], pos[t], xy)
        finished |= done
        if (t + 1) % check_every == 0 and bool(finished.all()):
            break
    fin = finished.cpu().numpy()
    rows_np = rows.cpu().numpy()
    xy_np = pos.cpu().numpy() if pos is not None else None
    if world > 1 and gather:
        parts = [None] * world
        dist.all_gather_object(parts, (offset, fin, rows_np, xy_np))
        parts.sort(key=lambda p: p[0])
        fin = np.concatenate([p[1] for p in parts])
        rows_np = np.concatenate([p[2] for p in parts])
        if xy_np is not None:
            T = max(p[3].shape[0] for p in parts)
            xy_np = np.concatenate([p[3][:T] for p in parts], 1)
    idx = np.flatnonzero(fin)
    recs = [info_dicts(r, nobs) for r in rows_np[idx]]
    out = {
        "successes": int(sum(d["n_successful_runs"] == 1 for d in recs)),
        "fails": int(sum(d["n_failed_runs"] == 1 for d in recs)),
        "collisions": np.array([d["n_collisions"] for d in recs], np.int64),
        "apes": np.array([d["APE"] for d in recs], np.float64),
        "time_spent": np.array([d["env_steps"] for d in recs], np.int64),
        "rewards": np.array([d["total_reward"] for d in recs], np.float64),
        "unfinished": int(len(fin) - len(recs)),
    }
    if xy_np is not None:
        steps = int(out["time_spent"].max()) if len(recs) else 0
        w, h = float(venv.kwargs["screensize_x"]), float(venv.kwargs["screensize_y"])
        xy = xy_np[:steps, idx].astype(np.float64)  # [steps, finished envs, 2]
        fl = np.stack([(xy[..., 0] + 1.0) * w / 2.0, h - (xy[..., 1] + 1.0) * h / 2.0], -1)
        fl[np.arange(steps)[:, None] >= out["time_spent"][None, :]] = np.nan  # after each episode's end
        out["flight_xy"] = fl
    return out


def write_results_rank0(m: dict, out_dir: str, scenario: str, agent_nr: str, agent_path: str):
    """``write_results`` on rank 0 only (a gathered ``run_first_episodes`` result); other ranks
    return None.  Without a process group it is ``write_results``."""
    _, rank, _ = _dist_world()
    return write_results(m, out_dir, scenario, agent_nr, agent_path) if rank == 0 else None


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


__all__ = ["MlpActor", "run_first_episodes", "flight_path_lists", "summary", "write_results",
           "write_results_rank0"]
