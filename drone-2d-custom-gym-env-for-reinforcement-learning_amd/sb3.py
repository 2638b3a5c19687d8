"""Stable-Baselines3 ``VecEnv`` adapter over the HIP batch.

The reference is trained with SB3 2.1 through ``SubprocVecEnv`` (main.py:88-101, 183-190): each
worker runs one ``Drone2dEnv`` (gym-0.21 API) behind shimmy's ``GymV21CompatibilityV0``, so the
learner sees ``VecEnv.step_wait() -> (obs[N,27] f32, rew[N], dones[N], infos)`` with

* ``dones = terminated | truncated`` where ``terminated`` is the env's ``done`` and ``truncated``
  is ``False`` (the reference never sets ``TimeLimit.truncated``; time-up is terminal),
* auto-reset: the returned row of a finished env is the first observation of its next episode and
  ``infos[i]["terminal_observation"]`` holds the last one,
* ``infos[i]`` = the reference's info dict (drone_2d_env.py:575-613) + ``"TimeLimit.truncated"``.

``SB3VecEnv`` reproduces that contract with the auto-reset done inside the step kernel.  When
stable_baselines3 is importable it is a real ``VecEnv`` subclass; otherwise a minimal base with the
same attributes and methods is used (SB3 is not installed in this image).

Building 65 536 info dicts per step costs far more than the step itself, so ``infos`` selects:
``"full"`` (the reference's dict for every env -- exact, slow), ``"done"`` (full dicts for finished
envs, ``{"TimeLimit.truncated": False}`` for the rest -- what SB3's Monitor/PPO read), ``"none"``
(only ``terminal_observation`` / ``TimeLimit.truncated``).  ``step_wait_tensors()`` is the
torch-native path (no host copies).
"""
from __future__ import annotations

import numpy as np
import torch

from . import abi
from .env import Drone2dVecEnv, info_dicts

try:  # pragma: no cover - SB3 is not installed in this image
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _VecEnvBase
except Exception:  # noqa: BLE001
    _VecEnvBase = None


class _MiniVecEnv:
    """The parts of ``stable_baselines3.common.vec_env.VecEnv`` (SB3 2.1) the learners use."""

    def __init__(self, num_envs, observation_space, action_space):
        self.num_envs = num_envs
        self.observation_space = observation_space
        self.action_space = action_space
        self.reset_infos = [{} for _ in range(num_envs)]
        self.render_mode = None

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def get_images(self):
        return []

    def render(self, mode=None):
        return None

    @property
    def unwrapped(self):
        return self

    def getattr_depth_check(self, name, already_found):
        return None


_Base = _VecEnvBase if _VecEnvBase is not None else _MiniVecEnv


class SB3VecEnv(_Base):
    """``VecEnv`` over ``num_envs`` HIP envs on one GPU (the reference's kwargs dict as ``**kwargs``)."""

    def __init__(self, num_envs: int, device=None, seed: int = 0, infos: str = "done", backend=None, **kwargs):
        """``backend``: an already-built batch with Drone2dVecEnv's interface (auto-reset on, info
        rows on); by default a Drone2dVecEnv is created from ``kwargs``."""
        if infos not in ("full", "done", "none"):
            raise ValueError("infos must be 'full', 'done' or 'none'")
        if backend is None:
            backend = Drone2dVecEnv(num_envs, device=device, seed=seed, auto_reset=True, with_info=True, **kwargs)
        self.venv = backend
        self.infos_mode = infos
        self._actions = None
        if _VecEnvBase is not None:  # pragma: no cover
            super().__init__(num_envs, self.venv.observation_space, self.venv.action_space)
        else:
            _MiniVecEnv.__init__(self, num_envs, self.venv.observation_space, self.venv.action_space)

    # ---------------------------------------------------------------- VecEnv API
    def reset(self):
        obs = self.venv.reset()
        self.reset_infos = [{} for _ in range(self.num_envs)]
        return obs.cpu().numpy()

    def step_async(self, actions):
        self._actions = actions

    def step_wait_tensors(self):
        """Torch-native step: (obs, rew, dones, terminated, truncated, terminal_obs, info) tensors."""
        obs, rew, term, trunc, info = self.venv.step(self._actions)
        return obs, rew, term | trunc, term, trunc, self.venv.terminal_obs, info

    def step_wait(self):
        obs, rew, dones, term, trunc, tobs, info = self.step_wait_tensors()
        obs_np = obs.cpu().numpy()
        rew_np = rew.cpu().numpy().astype(np.float32)
        dones_np = dones.cpu().numpy()
        trunc_np = trunc.cpu().numpy()
        idx = np.nonzero(dones_np)[0]
        tobs_np = tobs[torch.as_tensor(idx, device=tobs.device)].cpu().numpy() if len(idx) else None
        if self.infos_mode == "full":
            rows = info.cpu().numpy()
            infos = [info_dicts(rows[i]) for i in range(self.num_envs)]
            for d in infos:
                d["TimeLimit.truncated"] = False  # set below for finished envs (truncated and not terminated)
        else:
            infos = [{"TimeLimit.truncated": False} for _ in range(self.num_envs)]
            if self.infos_mode == "done" and len(idx):
                rows = info[torch.as_tensor(idx, device=info.device)].cpu().numpy()
                for k, i in enumerate(idx):
                    infos[i] = info_dicts(rows[k])
        for k, i in enumerate(idx):
            infos[i]["TimeLimit.truncated"] = bool(trunc_np[i])
            infos[i]["terminal_observation"] = tobs_np[k]
        return obs_np, rew_np, dones_np, infos

    def close(self):
        self.venv.close()

    def seed(self, seed=None):
        if seed is not None:
            self.venv.seed_value = int(seed)
        return [self.venv.seed_value] * self.num_envs

    def get_attr(self, attr_name, indices=None):
        val = getattr(self.venv, attr_name)
        return [val for _ in self._indices(indices)]

    def set_attr(self, attr_name, value, indices=None):
        setattr(self.venv, attr_name, value)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        fn = getattr(self.venv, method_name)
        res = fn(*method_args, **method_kwargs)
        return [res for _ in self._indices(indices)]

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False for _ in self._indices(indices)]

    # ---------------------------------------------------------------- helpers
    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices


__all__ = ["SB3VecEnv", "abi"]
