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
    manual: bool = True             # MLP backward + Adam written out over flat buffers (ManualStep)

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


_PPO_LIB = None

import ctypes as _C  # noqa: E402


class D2DPPORollout(_C.Structure):
    """include/d2d_ppo.h ``d2d_ppo_rollout`` (one fused rollout step, ABI v4)."""
    _fields_ = [(k, _C.c_int32) for k in ("n", "t", "T", "info_dim", "info_totrew")] + \
               [("gamma", _C.c_float), ("gae_lambda_gamma", _C.c_float), ("pad", _C.c_int32)] + \
               [(k, _C.c_void_p) for k in ("obs", "noise", "log_std", "prev_rew", "prev_term", "prev_trunc",
                                           "prev_info", "obs_buf", "act_buf", "logp_buf", "val_buf", "rew_buf",
                                           "done_buf", "start0", "act_env", "adv_buf", "ret_buf", "stats")]


def ppo_native():
    """ctypes binding of libd2d_ppo.so (include/d2d_ppo.h), loaded once; no fallback on a GPU."""
    global _PPO_LIB
    if _PPO_LIB is None:
        import ctypes as C
        import os

        from . import _native  # noqa: F401  (torch owns the HIP runtime first)

        path = os.environ.get("D2D_PPO_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                             "libd2d_ppo.so")  # (env: A/B builds, tools/)
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not found: the HIP extension is not built "
                               "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
        lib = C.CDLL(path)
        vp, i32, i64, f32 = C.c_void_p, C.c_int32, C.c_int64, C.c_float
        sig = {
            "d2d_ppo_abi_version": [],
            "d2d_ppo_adv_stats": [i32, vp, vp, vp, vp],
            "d2d_ppo_head_finish": [i32, i32, vp, vp, f32, vp, vp, vp, vp, vp, vp],
            "d2d_ppo_adam": [i32, vp, vp, vp, vp, vp, f32, f32, f32, f32, f32, vp],
            "d2d_ppo_wgrad": [i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp, vp],
            "d2d_ppo_wgrad_head": [i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp,
                                   i32, vp, vp, f32, vp, vp, vp, vp, vp, vp],
            "d2d_ppo_wgrad_chunks": [i32],
            "d2d_ppo_mlp_forward": [i32, vp, vp, vp, vp, vp, vp],
            "d2d_ppo_mlp_forward_adv": [i32, vp, vp, vp, vp, vp, vp, vp, vp],
            "d2d_ppo_mlp_backward": [i32, vp, vp, vp, vp, vp, vp, vp, i32, f32, f32, vp, vp, vp, vp, vp],
            "d2d_ppo_mlp_partial_rows": [i32],
            "d2d_ppo_permute": [i64, i32, C.c_uint64, vp, vp, vp],
            "d2d_ppo_rollout_step": [C.POINTER(D2DPPORollout), vp, vp],
            "d2d_ppo_fused_rows": [i32],
            "d2d_ppo_fused_grad": [i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, f32, f32, vp, vp, i32, vp, vp, vp],
            "d2d_ppo_grad_reduce": [i32, i32, vp, vp, i32, vp, i32, vp, f32, vp, vp, vp, vp, vp, vp],
        }
        for name, args in sig.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = C.c_int32, args
        if lib.d2d_ppo_abi_version() != 6:
            raise RuntimeError("libd2d_ppo.so ABI mismatch")
        _PPO_LIB = lib
    return _PPO_LIB


def _ok(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what}: hipError {rc}")


def _wgrad(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, rows: int = 512):
    """out = a^T b for a [M, p], b [M, q] (a weight gradient: the sum over the minibatch's samples).
    With K = M in the tens of thousands and a tiny p x q output, one GEMM runs on a handful of
    workgroups; split the sample axis into M / rows chunks (one batched GEMM) and add them up."""
    M = a.shape[0]
    if M % rows or M < 4 * rows:
        torch.mm(a.t(), b, out=out)
        return
    S = M // rows
    torch.sum(torch.bmm(a.reshape(S, rows, a.shape[1]).transpose(1, 2), b.reshape(S, rows, b.shape[1])), 0, out=out)


class ManualStep:
    """One SB3 PPO minibatch step (``PPO._minibatch``'s loss, gradient, clipping and Adam) with the
    backward pass of the two 27-64-64 tanh MLPs written out instead of recorded by autograd, over
    flat parameter / gradient / Adam-moment buffers (the module's parameters become views of them),
    and nothing that waits for the host -- the whole step captures into one HIP graph.  On a GPU
    it is seven libd2d_ppo.so launches (advantage statistics, both MLPs forward with four threads per
    sample and net, loss head + backward to the hidden-layer gradients, all weight / bias gradients
    + their reduce, log_std's gradient and the statistics, clip + Adam) instead of ~190 autograd /
    optimiser kernels; on the CPU the same math in torch ops (split-K weight gradients).

    Gradients of the loss (SB3 PPO.train, stable_baselines3/ppo/ppo.py 2.1):
      ratio = exp(logp - old_logp), s1 = adv ratio, s2 = adv clamp(ratio, 1 - c, 1 + c)
      d(-mean min(s1, s2)) / d logp_i = -adv_i [s1_i <= s2_i] ratio_i / M   (ties: autograd splits
        the gradient between the two equal branches, whose derivatives are then both adv_i)
      d logp / d mean = z / sigma, d logp / d log_std = z^2 - 1 (z = (a - mean) / sigma);
      entropy bonus: d(-ent_coef mean H) / d log_std = -ent_coef; value: vf_coef * -2 (R - V) / M.
    Adam as torch.optim.Adam (lerp first moment, bias corrections, eps outside the square root)."""

    def __init__(self, policy: ActorCritic, cfg: PPOConfig, device):
        self.pol, self.cfg = policy, cfg
        params = list(policy.parameters())
        n = sum(p.numel() for p in params)
        self.P = torch.zeros(n, device=device)
        self.G = torch.zeros(n, device=device)
        self.m = torch.zeros(n, device=device)
        self.v = torch.zeros(n, device=device)
        self.t = torch.zeros((), device=device)
        # the fused element-wise kernels on a GPU (libd2d_ppo.so, loud if missing); torch ops on CPU
        self.lib = ppo_native() if torch.device(device).type == "cuda" else None
        self._bufs = {}  # minibatch size -> (work buffers, partial rows) of the HIP path
        import os

        # D2D_PPO_FUSED=1 (default): forward + backward + weight gradients in one launch
        # (d2d_ppo_fused_grad) + the reduce; 0: the separate kernels (forward, backward, wgrad + reduce)
        self.fused = self.lib is not None and os.environ.get("D2D_PPO_FUSED", "1") == "1"
        o = 0
        for p in params:
            k = p.numel()
            self.P[o:o + k].copy_(p.data.reshape(-1))
            p.data = self.P[o:o + k].view_as(p)
            p.grad = self.G[o:o + k].view_as(p)
            o += k

    def step(self, idx, rollout, acc: dict, world: int = 1, adv_ws=None):
        self.grad(idx, rollout, acc, adv_ws)
        self.apply(world)

    def grad(self, idx, rollout, acc: dict, adv_ws=None):
        """The loss gradient of minibatch ``idx`` of ``rollout`` = (obs, actions, old log-probs,
        advantages, returns) into ``G``; statistics added to ``acc``."""
        cfg, pol = self.cfg, self.pol
        pn, vn = pol.mlp_extractor.policy_net, pol.mlp_extractor.value_net
        W1p, W2p, W1v, W2v = pn[0].weight, pn[2].weight, vn[0].weight, vn[2].weight
        W3p, W3v, ls = pol.action_net.weight, pol.value_net.weight, pol.log_std
        obs_all, act_all, ol_all, adv_all, ret_all = rollout
        if self.lib is not None:
            if self.fused:
                self._grad_fused(idx, rollout, acc, adv_ws)
            else:
                self._grad_hip(idx, rollout, acc)
            return
        X = obs_all[idx]
        M, c = X.shape[0], cfg.clip_range
        # forward (nn.Linear = addmm)
        h1p = torch.tanh(torch.addmm(pn[0].bias, X, W1p.t()))
        h2p = torch.tanh(torch.addmm(pn[2].bias, h1p, W2p.t()))
        mean = torch.addmm(pol.action_net.bias, h2p, W3p.t())
        h1v = torch.tanh(torch.addmm(vn[0].bias, X, W1v.t()))
        h2v = torch.tanh(torch.addmm(vn[2].bias, h1v, W2v.t()))
        V = torch.addmm(pol.value_net.bias, h2v, W3v.t()).squeeze(1)
        g_mean, g_V = self._head_torch(mean, V, act_all[idx], ol_all[idx], adv_all[idx], ret_all[idx], acc)
        tg = self._tanh_grad_torch
        # backward: the layer-output gradients, then every weight / bias gradient
        g2p = tg(h2p, torch.mm(g_mean, W3p))
        g2v = tg(h2v, g_V[:, None] * W3v)
        g1p = tg(h1p, torch.mm(g2p, W2p))
        g1v = tg(h1v, torch.mm(g2v, W2v))
        layers = ((g_mean, h2p, pol.action_net), (g_V[:, None], h2v, pol.value_net), (g2p, h1p, pn[2]),
                  (g2v, h1v, vn[2]), (g1p, X, pn[0]), (g1v, X, vn[0]))
        for a, b, lin in layers:
            _wgrad(a, b, lin.weight.grad)
            torch.sum(a, 0, out=lin.bias.grad)

    def _grad_hip(self, idx, rollout, acc):
        """libd2d_ppo.so: advantage statistics, both MLPs forward (four threads per sample and net),
        loss head + backward to the hidden-layer gradients, all weight / bias gradients, log_std's."""
        import ctypes as C

        cfg, pol, lib, st = self.cfg, self.pol, self.lib, self._stream()
        obs_all, act_all, ol_all, adv_all, ret_all = rollout
        M, dev = idx.numel(), self.P.device
        nb = (M + 63) // 64  # D2D_PPO_HEAD_BLOCK rows per advantage partial
        if M not in self._bufs:
            # one set of work buffers per minibatch size, kept for the handle's life: a captured graph
            # holds the full-size set's addresses while a ragged last minibatch runs eagerly on its own
            e = lambda *sh: torch.empty(*sh, device=dev)  # noqa: E731
            hb = {"h1p": e(M, 64), "h2p": e(M, 64), "mean": e(M, 2), "g1p": e(M, 64), "g2p": e(M, 64),
                  "h1v": e(M, 64), "h2v": e(M, 64), "val": e(M, 1), "g1v": e(M, 64), "g2v": e(M, 64),
                  "xg": e(M, 27), "gm": e(M, 2), "gv": e(M, 1),
                  "ws": torch.zeros(nb, 2, dtype=torch.float64, device=dev)}
            prow = lib.d2d_ppo_mlp_partial_rows(M)
            hb["partial"] = torch.zeros(prow, 5, device=dev)
            hb["wpart"] = e(lib.d2d_ppo_wgrad_chunks(M) * self.G.numel())  # weight-gradient partial rows
            self._bufs[M] = (hb, prow)
        hb, prow = self._bufs[M]
        pn, vn = pol.mlp_extractor.policy_net, pol.mlp_extractor.value_net
        wptr = self.weight_ptrs()
        bptr = (C.c_void_p * 10)(*[hb[k].data_ptr() for k in ("h1p", "h2p", "mean", "g1p", "g2p",
                                                              "h1v", "h2v", "val", "g1v", "g2v")])
        gptr = (C.c_void_p * 2)(hb["gm"].data_ptr(), hb["gv"].data_ptr())
        norm = int(cfg.normalize_advantage and M > 1)
        # the forward launch also writes the advantage statistics' partials when they are needed
        _ok(lib.d2d_ppo_mlp_forward_adv(M, idx.data_ptr(), obs_all.data_ptr(), adv_all.data_ptr() if norm else None,
                                        wptr, bptr, hb["xg"].data_ptr(), hb["ws"].data_ptr(), st),
            "d2d_ppo_mlp_forward_adv")
        _ok(lib.d2d_ppo_mlp_backward(M, idx.data_ptr(), act_all.data_ptr(), ol_all.data_ptr(), adv_all.data_ptr(),
                                     ret_all.data_ptr(), pol.log_std.data_ptr(), hb["ws"].data_ptr(), norm,
                                     cfg.clip_range, cfg.vf_coef, wptr, bptr, gptr, hb["partial"].data_ptr(), st),
            "d2d_ppo_mlp_backward")
        layers = ((hb["gm"], hb["h2p"], pol.action_net), (hb["gv"], hb["h2v"], pol.value_net),
                  (hb["g2p"], hb["h1p"], pn[2]), (hb["g2v"], hb["h1v"], vn[2]), (hb["g1p"], hb["xg"], pn[0]),
                  (hb["g1v"], hb["xg"], vn[0]))
        ls = pol.log_std
        # the head's finish (log-std gradient, loss statistics) rides on the gradient reduce's launch
        head = (prow, hb["partial"].data_ptr(), ls.data_ptr(), cfg.ent_coef, ls.grad.data_ptr(),
                acc["policy_loss"].data_ptr(), acc["value_loss"].data_ptr(), acc["entropy"].data_ptr(),
                acc["clip_fraction"].data_ptr())
        self._wgrad_hip(M, layers, hb["wpart"], head)

    def _grad_fused(self, idx, rollout, acc, adv_ws=None):
        """libd2d_ppo.so, two launches (+ the advantage statistics unless ``adv_ws`` points at this
        minibatch's precomputed d2d_ppo_adv_stats partials): d2d_ppo_fused_grad (both MLPs forward,
        the loss head, the backward and every weight / bias gradient, per-sample state on chip) and
        d2d_ppo_grad_reduce (the workgroups' rows into G, log_std's gradient, statistics)."""
        import ctypes as C

        cfg, pol, lib, st = self.cfg, self.pol, self.lib, self._stream()
        obs_all, act_all, ol_all, adv_all, ret_all = rollout
        M, dev = idx.numel(), self.P.device
        key = ("fused", M)
        if key not in self._bufs:
            rows = lib.d2d_ppo_fused_rows(M)
            nb = (M + 63) // 64
            self._bufs[key] = {"rows": rows, "wpart": torch.empty(rows * self.G.numel(), device=dev),
                               "hpart": torch.empty(2 * rows * 5, device=dev),
                               "ws": torch.zeros(nb, 2, dtype=torch.float64, device=dev)}
        b = self._bufs[key]
        pn, vn = pol.mlp_extractor.policy_net, pol.mlp_extractor.value_net
        base = self.G.data_ptr()
        layers = (pn[0], pn[2], pol.action_net, vn[0], vn[2], pol.value_net)
        offs = []
        for k in range(2):
            for lin in layers[3 * k:3 * k + 3]:
                offs += [(lin.weight.grad.data_ptr() - base) // 4, (lin.bias.grad.data_ptr() - base) // 4]
        offsets = (C.c_int32 * 12)(*offs)
        norm = int(cfg.normalize_advantage and M > 1)
        ws = adv_ws if adv_ws is not None else b["ws"].data_ptr()
        if norm and adv_ws is None:
            _ok(lib.d2d_ppo_adv_stats(M, idx.data_ptr(), adv_all.data_ptr(), ws, st), "d2d_ppo_adv_stats")
        _ok(lib.d2d_ppo_fused_grad(M, idx.data_ptr(), obs_all.data_ptr(), act_all.data_ptr(), ol_all.data_ptr(),
                                   adv_all.data_ptr(), ret_all.data_ptr(), pol.log_std.data_ptr(), ws,
                                   norm, cfg.clip_range, cfg.vf_coef, self.weight_ptrs(), offsets, self.G.numel(),
                                   b["wpart"].data_ptr(), b["hpart"].data_ptr(), st), "d2d_ppo_fused_grad")
        ls = pol.log_std
        _ok(lib.d2d_ppo_grad_reduce(b["rows"], self.G.numel(), b["wpart"].data_ptr(), base, 2 * b["rows"],
                                    b["hpart"].data_ptr(), M, ls.data_ptr(), cfg.ent_coef, ls.grad.data_ptr(),
                                    acc["policy_loss"].data_ptr(), acc["value_loss"].data_ptr(),
                                    acc["entropy"].data_ptr(), acc["clip_fraction"].data_ptr(), st),
            "d2d_ppo_grad_reduce")

    def weight_ptrs(self):
        """The 12 weight / bias device pointers of include/d2d_ppo.h (policy net, then value net);
        views of the flat parameter buffer, so the addresses never change."""
        import ctypes as C

        pol = self.pol
        pn, vn = pol.mlp_extractor.policy_net, pol.mlp_extractor.value_net
        ws = [pn[0].weight, pn[0].bias, pn[2].weight, pn[2].bias, pol.action_net.weight, pol.action_net.bias,
              vn[0].weight, vn[0].bias, vn[2].weight, vn[2].bias, pol.value_net.weight, pol.value_net.bias]
        return (C.c_void_p * 12)(*[w.data_ptr() for w in ws])

    @staticmethod
    def _tanh_grad_torch(h, g):
        return g.mul_(1.0 - h * h)

    def _wgrad_hip(self, M, layers, wpart, head=None):
        """All six weight / bias gradients in one libd2d_ppo.so launch (+ its reduce) into G; with
        `head` (d2d_ppo_head_finish's arguments after m) the reduce launch also finishes the head."""
        import ctypes as C

        row_len = self.G.numel()  # all of G: log_std's slots (no problem covers them) are rewritten after
        assert wpart.numel() >= self.lib.d2d_ppo_wgrad_chunks(M) * row_len
        n = len(layers)
        base = self.G.data_ptr()
        arr = lambda ty, v: (ty * n)(*v)  # noqa: E731
        a_p = arr(C.c_void_p, [a.data_ptr() for a, _, _ in layers])
        b_p = arr(C.c_void_p, [b.data_ptr() for _, b, _ in layers])
        lda = arr(C.c_int32, [a.stride(0) for a, _, _ in layers])
        ldb = arr(C.c_int32, [b.stride(0) for _, b, _ in layers])
        pp = arr(C.c_int32, [a.shape[1] for a, _, _ in layers])
        qq = arr(C.c_int32, [b.shape[1] for _, b, _ in layers])
        wo = arr(C.c_int32, [(lin.weight.grad.data_ptr() - base) // 4 for _, _, lin in layers])
        bo = arr(C.c_int32, [(lin.bias.grad.data_ptr() - base) // 4 for _, _, lin in layers])
        for a, b, _ in layers:
            assert a.stride(1) == 1 and b.stride(1) == 1 and a.shape[0] == b.shape[0] == M
        if head is None:
            _ok(self.lib.d2d_ppo_wgrad(M, n, a_p, lda, b_p, ldb, pp, qq, wo, bo, row_len, wpart.data_ptr(), base,
                                       self._stream()), "d2d_ppo_wgrad")
        else:
            _ok(self.lib.d2d_ppo_wgrad_head(M, n, a_p, lda, b_p, ldb, pp, qq, wo, bo, row_len, wpart.data_ptr(), base,
                                            *head, self._stream()), "d2d_ppo_wgrad_head")

    def _stream(self):
        return torch.cuda.current_stream(self.P.device).cuda_stream

    def _head_torch(self, mean, V, A, OL, ADV, R, acc):
        cfg, ls = self.cfg, self.pol.log_std
        M, c = mean.shape[0], cfg.clip_range
        isig = torch.exp(-ls)
        z = (A - mean) * isig
        logp = (-0.5 * z * z - ls - _HALF_LOG_2PI).sum(1)
        adv = ADV
        if cfg.normalize_advantage and M > 1:
            adv = (ADV - ADV.mean()) / (ADV.std() + 1e-8)
        ratio = torch.exp(logp - OL)
        s1 = adv * ratio
        s2 = adv * torch.clamp(ratio, 1 - c, 1 + c)
        pl = -torch.minimum(s1, s2).mean()
        err = R - V
        vl = (err * err).mean()
        g_lp = torch.where(s1 <= s2, adv, 0.0) * ratio * (-1.0 / M)  # d loss / d logp
        gz = g_lp[:, None] * z
        g_mean = gz * isig
        g_V = err * (-2.0 * cfg.vf_coef / M)
        torch.sum(gz * z - g_lp[:, None], 0, out=ls.grad)
        ls.grad.sub_(cfg.ent_coef)
        acc["policy_loss"] += pl
        acc["value_loss"] += vl
        acc["entropy"] += (0.5 + _HALF_LOG_2PI + ls).sum()
        acc["clip_fraction"] += ((ratio - 1).abs() > c).float().mean()
        return g_mean, g_V

    def apply(self, world: int = 1):
        """Rank-mean of ``G`` (RCCL), clip_grad_norm_, Adam step on ``P``."""
        cfg, G = self.cfg, self.G
        if world > 1:
            dist.all_reduce(G)  # data-parallel PPO: mean gradient over the ranks (RCCL)
            G.div_(world)
        if self.lib is not None:
            _ok(self.lib.d2d_ppo_adam(G.numel(), self.P.data_ptr(), G.data_ptr(), self.m.data_ptr(),
                                      self.v.data_ptr(), self.t.data_ptr(), cfg.learning_rate, 0.9, 0.999, 1e-5,
                                      cfg.max_grad_norm, self._stream()), "d2d_ppo_adam")
            return
        # clip_grad_norm_(max_grad_norm): scale by min(1, max / (||g|| + 1e-6))
        G.mul_(torch.clamp(cfg.max_grad_norm / (torch.linalg.vector_norm(G) + 1e-6), max=1.0))
        # Adam(lr, betas (0.9, 0.999), eps 1e-5)
        b1, b2, eps = 0.9, 0.999, 1e-5
        self.t.add_(1.0)
        self.m.lerp_(G, 1.0 - b1)
        self.v.mul_(b2).addcmul_(G, G, value=1.0 - b2)
        bc1 = 1.0 - torch.pow(b1, self.t)
        bc2s = torch.sqrt(1.0 - torch.pow(b2, self.t))
        self.P.sub_(self.m * (cfg.learning_rate / bc1) / (self.v.sqrt() / bc2s + eps))


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
        if self.world > 1:
            # one policy on every rank: rank 0's initial parameters; each rank its own noise stream
            for p in self.policy.parameters():
                dist.broadcast(p.data, 0)
        self.manual = ManualStep(self.policy, self.cfg, self.device) if self.cfg.manual else None
        self.opt = None if self.manual else torch.optim.Adam(self.policy.parameters(), lr=self.cfg.learning_rate,
                                                             eps=1e-5, capturable=self.use_graph)
        rank = dist.get_rank() if self.world > 1 else 0
        self.gen = torch.Generator(device=self.device).manual_seed(seed + 1_000_003 * rank)
        self.n_envs = int(venv.num_envs)
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
        self._ro = None          # rollout buffers (_alloc_rollout)
        self._ro_graph = None    # the captured rollout (GPU)
        self._ro_warm = False
        self._ro_gen = None      # the env's generation the rollout graph was captured against
        # the libd2d_ppo.so path (GPU, ManualStep): the epochs' shuffles from d2d_ppo_permute (a device
        # counter keys them, so the whole update -- shuffles and every minibatch step -- replays as one
        # HIP graph) and the rollout as one fused launch per step (d2d_ppo_rollout_step)
        self._hip = self.manual is not None and self.manual.lib is not None
        self._perm = None
        self._perm_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self._perm_seed = (seed * 0x9E3779B97F4A7C15 + rank * 0xD1B54A32D192ED03 + 1) % (1 << 64)
        self._upd_warm = False
        self._adv_ws = None      # every minibatch's advantage-statistics partials (_train_body_hip)
        self._fused = None       # decided at the first rollout (_alloc_rollout)

    # ------------------------------------------------------------------ rollout
    def _alloc_rollout(self):
        from .env import Drone2dVecEnv

        T, N, dev = self.cfg.n_steps, self.n_envs, self.device
        f64 = dict(dtype=torch.float64, device=dev)
        # time-limit truncations are bootstrapped with V(terminal obs); the reference never truncates
        self._truncates = bool(getattr(getattr(self.venv, "cfg", None), "timeup_truncates", 1))
        # the fused rollout: the HIP env batch, no truncation bootstrap (its extra value pass stays in torch)
        self._fused = bool(self._hip and isinstance(self.venv, Drone2dVecEnv) and not self._truncates)
        self._ro = {"val": torch.empty(T, N, device=dev), "rew": torch.empty(T, N, device=dev),
                    "done": torch.empty(T, N, dtype=torch.bool, device=dev),
                    "start0": torch.empty(N, dtype=torch.bool, device=dev),
                    "noise": torch.empty(T, N, 2, device=dev), "fin": torch.zeros((), **f64),
                    "ret": torch.zeros((), **f64)}
        if self._fused:
            self._ro["act_env"] = torch.empty(N, 2, device=dev)
            self._ro["stats"] = torch.zeros(T, (N + 63) // 64, 2, **f64)
            self._ro["obs_cur"] = None
        else:
            self._ro.update(obs=torch.empty(T + 1, N, 27, device=dev), act=torch.empty(T, N, 2, device=dev),
                            logp=torch.empty(T, N, device=dev))

    def _set_first_obs(self, obs):
        if self._fused:
            self._ro["obs_cur"] = obs  # the env's output tensor; the fused step reads it in place
        else:
            self._ro["obs"][0].copy_(obs.to(self.device))
        self._ro["start0"].fill_(True)

    @torch.no_grad()
    def _rollout_body_fused(self):
        """_rollout_body as T + 1 libd2d_ppo.so launches around the T env steps: step t's launch runs
        both MLPs on the env's observation tensor, samples and stores the action, log-density and
        value, copies the observations into the flat buffer and records step t-1's reward / done /
        episode statistics; the last one adds the bootstrap value and GAE (d2d_ppo_rollout_step)."""
        import ctypes as C

        from . import abi

        R, T, N, lib = self._ro, self.cfg.n_steps, self.n_envs, self.manual.lib
        st = self.manual._stream()
        wptr = self.manual.weight_ptrs()
        obs_buf, act_buf, logp_buf, adv_buf, ret_buf = self._flat
        ptr = lambda x: x.data_ptr() if x is not None else None  # noqa: E731
        r = D2DPPORollout(n=N, T=T, info_dim=abi.INFO_DIM, info_totrew=abi.INFO_TOTREW, gamma=self.cfg.gamma,
                          gae_lambda_gamma=self.cfg.gamma * self.cfg.gae_lambda,
                          log_std=ptr(self.policy.log_std), obs_buf=ptr(obs_buf), act_buf=ptr(act_buf),
                          logp_buf=ptr(logp_buf), val_buf=ptr(R["val"]), rew_buf=ptr(R["rew"]),
                          done_buf=ptr(R["done"]), start0=ptr(R["start0"]), act_env=ptr(R["act_env"]),
                          adv_buf=ptr(adv_buf), ret_buf=ptr(ret_buf), stats=ptr(R["stats"]))
        obs = R["obs_cur"]
        for t in range(T + 1):
            r.t = t
            r.obs = ptr(obs)
            r.noise = ptr(R["noise"][t]) if t < T else None
            _ok(lib.d2d_ppo_rollout_step(C.byref(r), wptr, st), "d2d_ppo_rollout_step")
            if t < T:
                obs, rew, term, trunc, info = self.venv.step(R["act_env"])
                r.prev_rew, r.prev_term, r.prev_trunc, r.prev_info = ptr(rew), ptr(term), ptr(trunc), ptr(info)
        R["obs_cur"] = obs  # T even: the same double-buffer slot as at the start
        R["fin"].copy_(R["stats"][..., 0].sum())
        R["ret"].copy_(R["stats"][..., 1].sum())

    @torch.no_grad()
    def _rollout_body(self):
        """n_steps policy + env steps into the rollout buffers, then GAE into the flat buffers.
        Reads obs[0], start0 and noise; leaves the next rollout's obs[0] / start0 in place.  No host
        synchronisation: on a GPU the whole body is one captured HIP graph."""
        from . import abi

        R, pol, T, dev = self._ro, self.policy, self.cfg.n_steps, self.device
        std = pol.log_std.exp()
        for t in range(T):
            mean, value = pol(R["obs"][t])
            actions = mean + std * R["noise"][t]
            logp = pol.log_prob(mean, actions)
            # SB3 clips to the Box bounds for the env only; the buffer keeps the unclipped action
            new_obs, rew, term, trunc, info = self.venv.step(actions.clamp(-1.0, 1.0))
            rew = rew.to(dev).float()
            trunc = trunc.to(dev)
            done = term.to(dev) | trunc
            if self._truncates:
                tv = pol.predict_values(self.venv.terminal_obs.to(dev))
                rew = torch.where(trunc, rew + self.cfg.gamma * tv, rew)
            R["obs"][t + 1].copy_(new_obs)
            R["act"][t].copy_(actions)
            R["logp"][t].copy_(logp)
            R["val"][t].copy_(value)
            R["rew"][t].copy_(rew)
            R["done"][t].copy_(done)
            if info is not None:
                R["fin"] += done.sum()
                R["ret"] += torch.where(done, info[:, abi.INFO_TOTREW].to(dev).double(), 0.0).sum()
        last_values = pol.predict_values(R["obs"][T])
        starts = torch.cat([R["start0"][None], R["done"][:-1]])
        adv, ret = compute_gae(R["rew"], R["val"], starts, last_values, R["done"][T - 1], self.cfg.gamma,
                               self.cfg.gae_lambda)
        N = self.n_envs
        for dst, src in zip(self._flat, (R["obs"][:T].reshape(T * N, 27), R["act"].reshape(T * N, 2),
                                         R["logp"].reshape(-1), adv.reshape(-1), ret.reshape(-1))):
            dst.copy_(src)
        R["obs"][0].copy_(R["obs"][T])
        R["start0"].copy_(R["done"][T - 1])

    def collect_rollouts(self) -> dict:
        T, N = self.cfg.n_steps, self.n_envs
        gen = getattr(self.venv, "generation", None)
        if self._ro is not None and gen != self._ro_gen:
            # the env re-allocated its scenario tables (set_curriculum / set_scenarios): a captured
            # rollout would replay against freed memory, and the envs were reset -- drop the graph
            # and start the next rollout from a reset
            self._ro_graph = None
            self._ro_warm = False
            self._set_first_obs(self.venv.reset())
        self._ro_gen = gen
        if self._ro is None:
            self._alloc_rollout()
            self._set_first_obs(self.venv.reset())
        R = self._ro
        body = self._rollout_body_fused if self._fused else self._rollout_body
        R["fin"].zero_()
        R["ret"].zero_()
        torch.randn(R["noise"].shape, generator=self.gen, device=self.device, out=R["noise"])
        # capture only whole fill periods: d2d_step launches the reset-cache fill after every 16th
        # step, decided on the host, so a graph of another length would bake in a fill on every
        # replay or on none (still correct through the synchronous reset path, but slower)
        graph_ok = self.cfg.graph and self.device.type == "cuda" and T % 16 == 0
        if graph_ok and self._ro_graph is None and self._ro_warm:
            # second rollout: capture (the first one ran eagerly: library and allocator warm-up);
            # T even, so the env's double-buffered outputs are back at their start after a replay
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                body()
            self._ro_graph = g
        if self._ro_graph is not None:
            self._ro_graph.replay()
        else:
            body()
            self._ro_warm = True
        self.num_timesteps += T * N
        f, r = float(R["fin"]), float(R["ret"])
        return {"episodes": f, "mean_return": r / f if f else float("nan")}

    # ------------------------------------------------------------------ update
    def _minibatch(self, idx: torch.Tensor, zero_grad: bool = True, adv_ws=None):
        """One SB3 PPO gradient step on rollout samples ``idx`` (statistics accumulated on device)."""
        obs, act, old_logp, adv_all, ret = self._flat
        if self.manual is not None:
            with torch.no_grad():
                self.manual.step(idx, self._flat, self._acc, self.world, adv_ws)
            return
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
        if self.opt is not None:
            self.opt.zero_grad(set_to_none=True)  # backward inside the capture writes fresh gradients
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._minibatch(self._gidx, zero_grad=False)
        for k, v in saved.items():  # capture does not execute: nothing to undo, but keep the sums exact
            self._acc[k].copy_(v)
        self._graph = g

    def _train_body_hip(self):
        """One update on the libd2d_ppo.so path: the n_epochs shuffles in one launch
        (d2d_ppo_permute), then every minibatch step; nothing waits for the host, so on one rank the
        whole update is captured and replayed as one HIP graph."""
        M, bs, E = self._flat[0].shape[0], self.cfg.batch_size, self.cfg.n_epochs
        for v in self._acc.values():
            v.zero_()
        lib, st = self.manual.lib, self.manual._stream()
        _ok(lib.d2d_ppo_permute(M, E, self._perm_seed, self._perm_ctr.data_ptr(), self._perm.data_ptr(), st),
            "d2d_ppo_permute")
        # the advantage statistics of every minibatch of the update in one launch: 64-row partials over
        # the whole shuffle; minibatch boundaries fall on partial boundaries when M and bs are multiples
        # of 64, so each minibatch reads its own slice (otherwise each minibatch computes its own)
        ws = None
        if self.manual.fused and self.cfg.normalize_advantage and M % 64 == 0 and bs % 64 == 0:
            if self._adv_ws is None:
                self._adv_ws = torch.zeros(E * M // 64, 2, dtype=torch.float64, device=self.device)
            _ok(lib.d2d_ppo_adv_stats(E * M, self._perm.data_ptr(), self._flat[3].data_ptr(),
                                      self._adv_ws.data_ptr(), st), "d2d_ppo_adv_stats")
            ws = self._adv_ws
        for e in range(E):
            for s in range(0, M, bs):
                n = min(s + bs, M) - s
                aw = ws[(e * M + s) // 64:].data_ptr() if (ws is not None and n > 1) else None
                self._minibatch(self._perm[e * M + s:e * M + s + n], adv_ws=aw)

    def train(self) -> dict:
        M, bs = self._flat[0].shape[0], self.cfg.batch_size
        if self._hip:
            if self._perm is None:
                self._perm = torch.empty(self.cfg.n_epochs * M, dtype=torch.int64, device=self.device)
            if self.use_graph and self._graph is None and self._upd_warm:
                # second update: capture the whole update (the first ran eagerly: kernels loaded, every
                # minibatch size's work buffers allocated)
                torch.cuda.synchronize(self.device)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._train_body_hip()
                self._graph = g
            if self._graph is not None:
                self._graph.replay()
            else:
                self._train_body_hip()
                self._upd_warm = True
            n_upd = self.cfg.n_epochs * -(-M // bs)
            return {k: float(v) / n_upd for k, v in self._acc.items()}
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


__all__ = ["PPOConfig", "ActorCritic", "ManualStep", "PPO", "compute_gae"]
