"""PPO end-to-end on the device: the rollout, GAE and the clipped-surrogate
update all stay on the GPU next to the HIP env batch, with no per-env Python objects.

The reference trains with Stable-Baselines3 2.1 ``PPO("MlpPolicy", env)`` over 14 SubprocVecEnv
workers (main.py:181-210; hyperparameters in ``ppo_agents/PFCA_see_3_obs_17_90.zip:data``: n_steps
2048, batch_size 64, n_epochs 10, gamma 0.99, gae_lambda 0.95, clip_range 0.2, ent_coef 0.01
(rl_config.py:7), vf_coef 0.5, max_grad_norm 0.5, lr 3e-4).  SB3 is not installed in this image;
this module restates the parts of SB3 2.1 that a training run executes, in the same order:

* ``ActorCritic``: SB3's ``MlpPolicy`` for a Box action space -- separate policy and value MLPs
  27-64-64 (tanh), ``action_net`` 64->2, ``value_net`` 64->1, state-independent ``log_std``
  (init 0), orthogonal init (gains sqrt(2) / 0.01 / 1, zero biases).  Parameter names follow SB3's
  state_dict, so a ``policy.pth`` from an SB3 zip loads into it.
* ``collect_rollouts`` (SB3 ``OnPolicyAlgorithm.collect_rollouts``): Gaussian actions, clipped to
  the action space only for the env; the stored actions and log-probabilities are the unclipped
  ones; rewards of time-limit truncations are bootstrapped with V(terminal obs) (the reference
  never truncates: time-up is terminal, so this path is idle by default).
* ``compute_returns_and_advantage`` (SB3 ``RolloutBuffer``): GAE(lambda) with episode starts.
* ``train`` (SB3 ``PPO.train``): shuffled minibatches, per-minibatch advantage normalisation,
  clipped surrogate, MSE value loss, entropy bonus, grad-norm clipping, Adam(eps=1e-5).

At 65 536 envs a 2 048-step rollout would hold 134 M transitions, so GPU-scale runs shorten
n_steps and enlarge batch_size (``PPOConfig.gpu_defaults``); the update rule is unchanged.  With
``torch.distributed`` initialised (one process per GPU, each with its env shard,
``drone2d_amd.shard``), gradients are averaged over ranks before each optimiser step (RCCL).
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist
from torch import nn


@dataclass
class PPOConfig:
    n_steps: int = 2048
    batch_size: int = 64
    n_epochs: int = 10
    learning_rate: float = 3e-4
    gamma: float = 0.99
    gae_lambda: float = 0.95
    clip_range: float = 0.2
    ent_coef: float = 0.01          # rl_config.py:7
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    normalize_advantage: bool = True
    graph: bool = True              # GPU, one rank: the minibatch update replayed as one HIP graph

    @classmethod
    def gpu_defaults(cls, **over) -> "PPOConfig":
        """Short rollouts over many envs (65 536 x 16 = 1 M samples per update), big minibatches."""
        return cls(**dict(dict(n_steps=16, batch_size=32768), **over))


_HALF_LOG_2PI = 0.5 * math.log(2.0 * math.pi)


class ActorCritic(nn.Module):
    """SB3 2.1 ``MlpPolicy`` (net_arch pi=[64, 64], vf=[64, 64], tanh) for obs 27 -> action 2."""

    def __init__(self, obs_dim: int = 27, act_dim: int = 2, hidden: int = 64, log_std_init: float = 0.0):
        super().__init__()
        self.mlp_extractor = nn.Module()
        self.mlp_extractor.policy_net = nn.Sequential(nn.Linear(obs_dim, hidden), nn.Tanh(),
                                                      nn.Linear(hidden, hidden), nn.Tanh())
        self.mlp_extractor.value_net = nn.Sequential(nn.Linear(obs_dim, hidden), nn.Tanh(),
                                                     nn.Linear(hidden, hidden), nn.Tanh())
        self.action_net = nn.Linear(hidden, act_dim)
        self.value_net = nn.Linear(hidden, 1)
        self.log_std = nn.Parameter(torch.ones(act_dim) * log_std_init)
        # ActorCriticPolicy._build, ortho_init=True
        for mod, gain in ((self.mlp_extractor, math.sqrt(2)), (self.action_net, 0.01), (self.value_net, 1.0)):
            for m in mod.modules():
                if isinstance(m, nn.Linear):
                    nn.init.orthogonal_(m.weight, gain=gain)
                    m.bias.data.fill_(0.0)

    def forward(self, obs: torch.Tensor):
        mean = self.action_net(self.mlp_extractor.policy_net(obs))
        value = self.value_net(self.mlp_extractor.value_net(obs)).squeeze(-1)
        return mean, value

    def dist(self, mean: torch.Tensor) -> torch.distributions.Normal:
        return torch.distributions.Normal(mean, torch.ones_like(mean) * self.log_std.exp(), validate_args=False)

    def log_prob(self, mean: torch.Tensor, actions: torch.Tensor) -> torch.Tensor:
        """Diagonal-Gaussian log density summed over the action dims (SB3 DiagGaussianDistribution),
        written out so it captures into a HIP graph (torch.distributions validates on the host)."""
        z = (actions - mean) * torch.exp(-self.log_std)
        return (-0.5 * z * z - self.log_std - _HALF_LOG_2PI).sum(-1)

    def entropy(self, n: int) -> torch.Tensor:
        return (0.5 + _HALF_LOG_2PI + self.log_std).sum().expand(n)

    def evaluate_actions(self, obs: torch.Tensor, actions: torch.Tensor):
        mean, value = self(obs)
        return value, self.log_prob(mean, actions), self.entropy(obs.shape[0])

    @torch.no_grad()
    def predict_values(self, obs: torch.Tensor) -> torch.Tensor:
        return self(obs)[1]

    @classmethod
    def from_agent_npz(cls, path: str) -> "ActorCritic":
        """The actor of a shipped agent (tests/golden/agent_17_90.npz: SB3 names with '.' -> '_');
        the value net keeps its fresh init (the fixture holds the actor only)."""
        m = cls()
        with np.load(path, allow_pickle=False) as z:
            sd = {k: torch.as_tensor(z[k]) for k in z.files}
        names = {n.replace(".", "_"): n for n in m.state_dict()}
        m.load_state_dict({names[k]: v for k, v in sd.items()}, strict=False)
        return m


def compute_gae(rewards, values, episode_starts, last_values, last_dones, gamma, gae_lambda):
    """SB3 ``RolloutBuffer.compute_returns_and_advantage``: tensors [T, N] (episode_starts[t] = the
    env started a new episode at step t), last_* [N]; returns (advantages, returns)."""
    T = rewards.shape[0]
    adv = torch.zeros_like(rewards)
    last_gae = torch.zeros_like(last_values)
    for step in reversed(range(T)):
        if step == T - 1:
            next_non_terminal = 1.0 - last_dones.to(rewards.dtype)
            next_values = last_values
        else:
            next_non_terminal = 1.0 - episode_starts[step + 1].to(rewards.dtype)
            next_values = values[step + 1]
        delta = rewards[step] + gamma * next_values * next_non_terminal - values[step]
        last_gae = delta + gamma * gae_lambda * next_non_terminal * last_gae
        adv[step] = last_gae
    return adv, adv + values


class PPO:
    """PPO on a batched env with Drone2dVecEnv's tensor interface (``reset() -> obs``,
    ``step(actions) -> (obs, reward, terminated, truncated, info)``, ``terminal_obs``)."""

    def __init__(self, venv, config: PPOConfig | None = None, policy: ActorCritic | None = None, seed: int = 0,
                 device=None):
        self.venv = venv
        self.cfg = config or PPOConfig()
        self.device = torch.device(device) if device is not None else torch.device(venv.device)
        torch.manual_seed(seed)
        self.policy = (policy or ActorCritic()).to(self.device)
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.use_graph = bool(self.cfg.graph and self.device.type == "cuda" and self.world == 1)
        self.opt = torch.optim.Adam(self.policy.parameters(), lr=self.cfg.learning_rate, eps=1e-5,
                                    capturable=self.use_graph)
        if self.world > 1:
            # one policy on every rank: rank 0's initial parameters; each rank its own noise stream
            for p in self.policy.parameters():
                dist.broadcast(p.data, 0)
        rank = dist.get_rank() if self.world > 1 else 0
        self.gen = torch.Generator(device=self.device).manual_seed(seed + 1_000_003 * rank)
        self.n_envs = int(venv.num_envs)
        self._last_obs = None
        self._last_episode_starts = None
        self.num_timesteps = 0
        # the rollout lands in fixed buffers (a captured update reads them at fixed addresses)
        M = self.cfg.n_steps * self.n_envs
        dev = self.device
        self._flat = (torch.empty(M, 27, device=dev), torch.empty(M, 2, device=dev), torch.empty(M, device=dev),
                      torch.empty(M, device=dev), torch.empty(M, device=dev))
        z = torch.zeros((), device=dev)
        self._acc = {"policy_loss": z.clone(), "value_loss": z.clone(), "entropy": z.clone(),
                     "clip_fraction": z.clone()}
        self._graph = None
        self._gidx = None

    # ------------------------------------------------------------------ rollout
    @torch.no_grad()
    def collect_rollouts(self) -> dict:
        T, N, dev = self.cfg.n_steps, self.n_envs, self.device
        if self._last_obs is None:
            self._last_obs = self.venv.reset().to(dev).clone()
            self._last_episode_starts = torch.ones(N, dtype=torch.bool, device=dev)
        obs_b = torch.empty(T, N, 27, device=dev)
        act_b = torch.empty(T, N, 2, device=dev)
        logp_b = torch.empty(T, N, device=dev)
        val_b = torch.empty(T, N, device=dev)
        rew_b = torch.empty(T, N, device=dev)
        start_b = torch.empty(T, N, dtype=torch.bool, device=dev)
        finished = torch.zeros((), dtype=torch.float64, device=dev)
        ret_sum = torch.zeros((), dtype=torch.float64, device=dev)
        for t in range(T):
            obs = self._last_obs
            mean, value = self.policy(obs)
            std = self.policy.log_std.exp()
            actions = mean + std * torch.randn(mean.shape, device=dev, generator=self.gen)
            logp = self.policy.log_prob(mean, actions)
            clipped = actions.clamp(-1.0, 1.0)  # SB3 clips to the Box bounds for the env only
            new_obs, rew, term, trunc, info = self.venv.step(clipped)
            rew = rew.to(dev).float()
            trunc = trunc.to(dev)
            done = term.to(dev) | trunc
            if bool(trunc.any()):
                # time-limit truncation: bootstrap with the value of the terminal observation
                tv = self.policy.predict_values(self.venv.terminal_obs.to(dev))
                rew = torch.where(trunc, rew + self.cfg.gamma * tv, rew)
            obs_b[t] = obs
            act_b[t] = actions
            logp_b[t] = logp
            val_b[t] = value
            rew_b[t] = rew
            start_b[t] = self._last_episode_starts
            self._last_obs = new_obs.to(dev).clone()
            self._last_episode_starts = done
            if info is not None:
                from . import abi

                finished += done.sum()
                ret_sum += torch.where(done, info[:, abi.INFO_TOTREW].to(dev).double(), 0.0).sum()
        last_values = self.policy.predict_values(self._last_obs)
        adv, ret = compute_gae(rew_b, val_b, start_b, last_values, self._last_episode_starts, self.cfg.gamma,
                               self.cfg.gae_lambda)
        for dst, src in zip(self._flat, (obs_b.reshape(T * N, 27), act_b.reshape(T * N, 2), logp_b.reshape(-1),
                                         adv.reshape(-1), ret.reshape(-1))):
            dst.copy_(src)
        self.num_timesteps += T * N
        f, r = float(finished), float(ret_sum)
        return {"episodes": f, "mean_return": r / f if f else float("nan")}

    # ------------------------------------------------------------------ update
    def _minibatch(self, idx: torch.Tensor, zero_grad: bool = True):
        """One SB3 PPO gradient step on rollout samples ``idx`` (statistics accumulated on device)."""
        obs, act, old_logp, adv_all, ret = self._flat
        c = self.cfg.clip_range
        params = list(self.policy.parameters())
        values, logp, entropy = self.policy.evaluate_actions(obs[idx], act[idx])
        adv = adv_all[idx]
        if self.cfg.normalize_advantage and idx.numel() > 1:
            adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        ratio = torch.exp(logp - old_logp[idx])
        pl = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - c, 1 + c)).mean()
        vl = torch.nn.functional.mse_loss(ret[idx], values)
        el = -entropy.mean()
        loss = pl + self.cfg.ent_coef * el + self.cfg.vf_coef * vl
        if zero_grad:
            self.opt.zero_grad(set_to_none=False)
        loss.backward()
        if self.world > 1:
            # data-parallel PPO: average the gradients over the ranks (RCCL all-reduce)
            flat = torch.cat([p.grad.reshape(-1) for p in params])
            dist.all_reduce(flat)
            flat /= self.world
            o = 0
            for p in params:
                k = p.numel()
                p.grad.copy_(flat[o:o + k].view_as(p))
                o += k
        torch.nn.utils.clip_grad_norm_(params, self.cfg.max_grad_norm)
        self.opt.step()
        with torch.no_grad():
            self._acc["policy_loss"] += pl
            self._acc["value_loss"] += vl
            self._acc["entropy"] -= el
            self._acc["clip_fraction"] += ((ratio - 1).abs() > c).float().mean()

    def _capture(self):
        """Record one full-size minibatch step as a HIP graph: forward, backward, grad clipping and
        the (capturable) Adam step replay with no per-kernel launches from Python."""
        bs = self.cfg.batch_size
        self._gidx = torch.zeros(bs, dtype=torch.long, device=self.device)
        saved = {k: v.clone() for k, v in self._acc.items()}
        self.opt.zero_grad(set_to_none=True)  # backward inside the capture writes fresh gradients
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._minibatch(self._gidx, zero_grad=False)
        for k, v in saved.items():  # capture does not execute: nothing to undo, but keep the sums exact
            self._acc[k].copy_(v)
        self._graph = g

    def train(self) -> dict:
        M, bs = self._flat[0].shape[0], self.cfg.batch_size
        for v in self._acc.values():
            v.zero_()
        n_upd = 0
        warm = 0
        for _ in range(self.cfg.n_epochs):
            perm = torch.randperm(M, device=self.device, generator=self.gen)
            for s in range(0, M, bs):
                idx = perm[s:s + bs]
                if self.use_graph and idx.numel() == bs:
                    if self._graph is None and warm >= 3:
                        # capture after a few eager steps (lazy optimiser state, allocator warm-up)
                        torch.cuda.synchronize(self.device)
                        self._capture()
                    if self._graph is not None:
                        self._gidx.copy_(idx)
                        self._graph.replay()
                        n_upd += 1
                        continue
                    warm += 1
                self._minibatch(idx)
                n_upd += 1
        return {k: float(v) / max(n_upd, 1) for k, v in self._acc.items()}

    def learn(self, total_timesteps: int, log=None) -> list[dict]:
        """Alternate rollouts and updates until ``total_timesteps`` env steps (this rank)."""
        hist = []
        while self.num_timesteps < total_timesteps:
            t0 = time.perf_counter()
            ro = self.collect_rollouts()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            t1 = time.perf_counter()
            tr = self.train()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            t2 = time.perf_counter()
            rec = dict(ro, **tr, timesteps=self.num_timesteps, rollout_s=t1 - t0, train_s=t2 - t1,
                       env_steps_per_s=self.cfg.n_steps * self.n_envs / (t2 - t0))
            hist.append(rec)
            if log:
                log(rec)
        return hist


__all__ = ["PPOConfig", "ActorCritic", "PPO", "compute_gae"]
