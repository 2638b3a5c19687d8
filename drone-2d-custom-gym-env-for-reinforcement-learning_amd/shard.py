"""Multi-GPU sharding of the batched env.

Envs never interact (each has its own Space in the reference), so N envs split into contiguous
blocks, one per rank / GPU, with no collective on the step path.  Two things keep a sharded run
identical to one big batch:

* global env ids -- every rank passes ``env_id_offset`` so the Philox spawn stream of env i is keyed
  by its global id (``d2d_cfg.env_id_base``);
* the env -> scenario map is computed globally (``i mod n_scenarios`` for config 5's mixed batch)
  and sliced.

The only collective is one SUM all-reduce of the 8-double episode-statistics vector per logging
interval (``allreduce_stats``): RCCL (torch.distributed "nccl") on GPUs, gloo on CPU tensors.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """(offset, count) of rank's contiguous block; the first n_total % world ranks get one more."""
    if world <= 0 or not 0 <= rank < world or n_total < world:
        raise ValueError("need 0 <= rank < world <= n_total")
    base, rem = divmod(n_total, world)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def global_env_scenario(n_total: int, n_scenarios: int) -> np.ndarray:
    """Config 5's mixed batch: env i runs scenario i mod n_scenarios."""
    return (np.arange(n_total) % n_scenarios).astype(np.int32)


def shard_env_scenario(env_scenario_global, offset: int, count: int) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(env_scenario_global, dtype=np.int32)[offset:offset + count])


def init_process_group_from_env(backend: str | None = None):
    """torch.distributed.run environment -> (rank, world, local_rank); world 1 needs no init.
    Backend: "nccl" (RCCL) when a HIP device is present, else "gloo"."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def allreduce_stats(stats: torch.Tensor, group=None) -> torch.Tensor:
    """In-place SUM of the episode-statistics vector over ranks (no-op without a process group)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.SUM, group=group)
    return stats


def make_shard_venv(n_total: int, rank: int, world: int, *, device=None, seed: int = 0, with_info: bool = True,
                    exact_trig: bool = False, **kwargs):
    """This rank's Drone2dVecEnv of a global batch of n_total envs (scenario i mod n_scenarios
    for global env i, as one unsharded batch would assign it)."""
    from .env import Drone2dVecEnv, build_scenarios, is_fresh_curriculum

    offset, count = shard_range(n_total, world, rank)
    opt = dict(device=device, seed=seed, env_id_offset=offset, with_info=with_info, exact_trig=exact_trig)
    if is_fresh_curriculum(kwargs):  # per-episode device scenarios; the stage clock counts all ranks' envs
        return Drone2dVecEnv(count, envs_total=n_total, **opt, **kwargs)
    es = shard_env_scenario(global_env_scenario(n_total, len(build_scenarios(kwargs))), offset, count)
    return Drone2dVecEnv(count, env_scenario=es, **opt, **kwargs)


__all__ = ["shard_range", "global_env_scenario", "shard_env_scenario", "init_process_group_from_env",
           "allreduce_stats", "make_shard_venv"]
