"""PPO end-to-end on the batched env: SB3 2.1's algorithm restated in torch.

CPU: GAE against an independent per-env restatement of SB3's RolloutBuffer recursion, the policy
against the shipped agent's actor, a short training run on the oracle-backed batch (test
infrastructure).  GPU: a short run on the HIP batch."""
import numpy as np
import pytest
import torch

from oracle_backend import OracleVecBackend


def _kw(**over):
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    return dict(ENV_TRAIN_CONFIG, **over)


def test_gae_matches_per_env_recursion(d2):
    from drone2d_amd.ppo import compute_gae

    rng = np.random.default_rng(0)
    T, N, g, lam = 7, 5, 0.99, 0.95
    r = rng.normal(size=(T, N))
    v = rng.normal(size=(T, N))
    starts = rng.random((T, N)) < 0.2
    lv = rng.normal(size=N)
    ld = rng.random(N) < 0.3
    adv, ret = compute_gae(*(torch.as_tensor(x) for x in (r, v, starts, lv, ld)), g, lam)
    for n in range(N):
        gae = 0.0
        for t in reversed(range(T)):
            nv, nt = (lv[n], 1.0 - ld[n]) if t == T - 1 else (v[t + 1, n], 1.0 - starts[t + 1, n])
            gae = (r[t, n] + g * nv * nt - v[t, n]) + g * lam * nt * gae
            assert abs(adv[t, n].item() - gae) < 1e-12
            assert abs(ret[t, n].item() - (gae + v[t, n])) < 1e-12


def test_actor_matches_shipped_agent(d2):
    import os

    from conftest import GOLDEN
    from drone2d_amd.harness import MlpActor
    from drone2d_amd.ppo import ActorCritic

    path = os.path.join(GOLDEN, "agent_17_90.npz")
    ac, ref = ActorCritic.from_agent_npz(path), MlpActor.from_npz(path)
    obs = torch.randn(64, 27)
    torch.testing.assert_close(ac(obs)[0], ref(obs))
    torch.testing.assert_close(ac.log_std.detach(), ref.log_std)
    # SB3 state_dict names: a policy.pth loads as-is
    assert "mlp_extractor.policy_net.0.weight" in ac.state_dict() and "value_net.weight" in ac.state_dict()


def test_ppo_trains_on_oracle_batch(d2):
    from drone2d_amd.ppo import PPO, PPOConfig

    be = OracleVecBackend(32, seed=3, **_kw(scenario="corridor"))
    algo = PPO(be, PPOConfig(n_steps=8, batch_size=64, n_epochs=2), seed=0, device="cpu")
    before = [p.detach().clone() for p in algo.policy.parameters()]
    hist = algo.learn(2 * 8 * 32)
    assert algo.num_timesteps == 512 and len(hist) == 2
    for h in hist:
        for k in ("policy_loss", "value_loss", "entropy", "clip_fraction"):
            assert np.isfinite(h[k]), (k, h)
    assert any(not torch.equal(a, b) for a, b in zip(before, algo.policy.parameters()))
    be.close()


@pytest.mark.gpu
def test_ppo_on_hip_batch(d2):
    from drone2d_amd.ppo import PPO, PPOConfig

    venv = d2.Drone2dVecEnv(4096, seed=1, **_kw(scenario="corridor"))
    algo = PPO(venv, PPOConfig.gpu_defaults(n_steps=8, batch_size=8192, n_epochs=2), seed=0)
    hist = algo.learn(3 * 8 * 4096)
    assert len(hist) == 3 and all(np.isfinite(h["value_loss"]) for h in hist)
    assert hist[-1]["env_steps_per_s"] > 0
    venv.close()


@pytest.mark.gpu
@pytest.mark.parametrize("bs", [4096, 12288])
def test_ppo_graph_update_matches_eager(d2, bs):
    """The HIP-graph replayed minibatch step computes what the eager step computes (bs = 12288:
    every epoch ends with a ragged 8 192-sample minibatch that runs eagerly between replays)."""
    from drone2d_amd.ppo import PPO, PPOConfig

    params = []
    for graph in (False, True):
        venv = d2.Drone2dVecEnv(4096, seed=1, **_kw(scenario="corridor"))
        cfg = PPOConfig.gpu_defaults(n_steps=8, batch_size=bs, n_epochs=4 if bs > 4096 else 2)
        cfg.graph = graph
        algo = PPO(venv, cfg, seed=0)
        assert algo.use_graph == graph
        hist = algo.learn(8 * 4096)
        assert (algo._graph is not None) == graph and np.isfinite(hist[-1]["value_loss"])
        params.append([p.detach().clone() for p in algo.policy.parameters()])
        venv.close()
    for a, b in zip(*params):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


def _manual_vs_autograd(M, device):
    from drone2d_amd.ppo import ActorCritic, ManualStep, PPOConfig

    torch.manual_seed(0)
    ref = ActorCritic()
    with torch.no_grad():  # a policy away from its init (log_std != 0, larger action head)
        ref.log_std.copy_(torch.tensor([-0.3, 0.2]))
        ref.action_net.weight.mul_(30.0)
    man = ActorCritic()
    man.load_state_dict(ref.state_dict())
    man = man.to(device)
    cfg = PPOConfig()
    g = torch.Generator().manual_seed(1)
    X = torch.randn(M, 27, generator=g) * 0.5
    A = torch.randn(M, 2, generator=g)
    ADV = torch.randn(M, generator=g)
    R = torch.randn(M, generator=g) * 3
    with torch.no_grad():
        mean, _ = ref(X)
        OL = ref.log_prob(mean, A) + torch.randn(M, generator=g) * 0.3  # ratios on both sides of the clip
    # autograd reference (PPO._minibatch's loss), on the CPU
    opt = torch.optim.Adam(ref.parameters(), lr=cfg.learning_rate, eps=1e-5)
    values, logp, ent = ref.evaluate_actions(X, A)
    adv = (ADV - ADV.mean()) / (ADV.std() + 1e-8)
    ratio = torch.exp(logp - OL)
    c = cfg.clip_range
    pl = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - c, 1 + c)).mean()
    vl = torch.nn.functional.mse_loss(R, values)
    loss = pl + cfg.ent_coef * (-ent.mean()) + cfg.vf_coef * vl
    loss.backward()
    grads = [p.grad.clone() for p in ref.parameters()]
    torch.nn.utils.clip_grad_norm_(list(ref.parameters()), cfg.max_grad_norm)
    opt.step()
    # manual (the fused HIP kernels on a GPU, torch ops on the CPU); rollout rows in shuffled order
    step = ManualStep(man, cfg, device)
    assert (step.lib is not None) == (torch.device(device).type == "cuda")
    perm = torch.randperm(M, generator=g)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(M)
    rollout = tuple(t[inv].contiguous().to(device) for t in (X, A, OL, ADV, R))  # row inv[i] -> sample i
    idx = perm.to(device)
    acc = {k: torch.zeros((), device=device) for k in ("policy_loss", "value_loss", "entropy", "clip_fraction")}
    with torch.no_grad():
        step.grad(idx, rollout, acc)
        for (name, p), gr in zip(man.named_parameters(), grads):
            torch.testing.assert_close(p.grad.cpu(), gr, rtol=2e-4, atol=1e-7, msg=name)
        step.apply()
    frac = float(((ratio - 1).abs() > c).float().mean())
    assert 0.05 < frac < 0.95  # both clip branches exercised
    for (name, p), q in zip(man.named_parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach().cpu(), q.detach(), rtol=1e-4, atol=1e-6, msg=name)
    torch.testing.assert_close(acc["policy_loss"].cpu(), pl.detach(), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(acc["value_loss"].cpu(), vl.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(acc["entropy"].cpu(), ent.mean().detach(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(acc["clip_fraction"].cpu(), torch.tensor(frac), rtol=0, atol=1e-7)


@pytest.mark.parametrize("M", [64, 4096])
def test_manual_step_matches_autograd(d2, M):
    """ManualStep's written-out backward + clipping + Adam against autograd + clip_grad_norm_ +
    torch.optim.Adam on the same minibatch (M = 4096 takes the split-K weight-gradient path)."""
    _manual_vs_autograd(M, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("M", [64, 1000, 32768])
def test_manual_step_hip_matches_autograd(d2, M):
    """The same with libd2d_ppo.so's fused head / tanh-backward / Adam kernels on the GPU."""
    _manual_vs_autograd(M, "cuda")


@pytest.mark.gpu
def test_fused_adam_matches_separate_launch(d2):
    """d2d_ppo_wgrad_head_adam (Adam as the gradient reduce's last workgroup) against the separate
    d2d_ppo_adam launch: parameters, moments, step counter, clipped gradient and loss statistics bit
    for bit over consecutive minibatches of different sizes (the device ticket resets itself)."""
    from drone2d_amd.ppo import ActorCritic, ManualStep, PPOConfig

    torch.manual_seed(3)
    base = ActorCritic()
    cfg = PPOConfig()
    g = torch.Generator().manual_seed(5)
    T = 40000
    rollout = tuple(t.cuda() for t in (torch.randn(T, 27, generator=g) * 0.5, torch.randn(T, 2, generator=g),
                                       torch.randn(T, generator=g) - 3.0, torch.randn(T, generator=g),
                                       torch.randn(T, generator=g) * 3))
    runs = []
    for fuse in (False, True):
        pol = ActorCritic()
        pol.load_state_dict(base.state_dict())
        step = ManualStep(pol.cuda(), cfg, "cuda")
        step.fuse_adam = fuse
        acc = {k: torch.zeros((), device="cuda") for k in ("policy_loss", "value_loss", "entropy", "clip_fraction")}
        gi = torch.Generator().manual_seed(7)
        with torch.no_grad():
            for M in (32768, 1000, 64, 32768, 7232):
                step.step(torch.randperm(T, generator=gi)[:M].cuda(), rollout, acc)
        torch.cuda.synchronize()
        assert int(step._ticket.item()) == 0
        runs.append([step.P, step.m, step.v, step.t, step.G] + [acc[k] for k in sorted(acc)])
    assert float(runs[0][3]) == 5.0
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_spread_adam_matches_one_workgroup(d2):
    """d2d_ppo_adam_spread (the Adam step over ~11 workgroups, step counter advanced by the last one
    through a device ticket) against d2d_ppo_adam over consecutive minibatches: same step count,
    parameters and moments equal up to the norm's summation order."""
    from drone2d_amd.ppo import ActorCritic, ManualStep, PPOConfig

    torch.manual_seed(4)
    base = ActorCritic()
    cfg = PPOConfig()
    g = torch.Generator().manual_seed(6)
    T = 40000
    rollout = tuple(t.cuda() for t in (torch.randn(T, 27, generator=g) * 0.5, torch.randn(T, 2, generator=g),
                                       torch.randn(T, generator=g) - 3.0, torch.randn(T, generator=g),
                                       torch.randn(T, generator=g) * 3))
    runs = []
    for spread in (False, True):
        pol = ActorCritic()
        pol.load_state_dict(base.state_dict())
        step = ManualStep(pol.cuda(), cfg, "cuda")
        step.fuse_adam, step.adam_spread = False, spread
        acc = {k: torch.zeros((), device="cuda") for k in ("policy_loss", "value_loss", "entropy", "clip_fraction")}
        gi = torch.Generator().manual_seed(8)
        with torch.no_grad():
            for M in (32768, 1000, 64, 32768, 7232):
                step.step(torch.randperm(T, generator=gi)[:M].cuda(), rollout, acc)
        torch.cuda.synchronize()
        assert int(step._ticket.item()) == 0
        assert float(step.t) == 5.0
        runs.append((step.P.cpu(), step.m.cpu(), step.v.cpu()))
    for a, b in zip(*runs):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_rollout_graph_matches_eager(d2):
    """The captured rollout (policy + env step + GAE replayed as one HIP graph) fills the same
    buffers as the eager loop, bit for bit, over three consecutive rollouts."""
    from drone2d_amd.ppo import PPO, PPOConfig

    outs = []
    for graph in (False, True):
        venv = d2.Drone2dVecEnv(2048, seed=4, with_info=True, **_kw(scenario="corridor"))
        cfg = PPOConfig.gpu_defaults(n_steps=16, batch_size=4096)
        cfg.graph = graph
        algo = PPO(venv, cfg, seed=2)
        rec = []
        for _ in range(3):
            st = algo.collect_rollouts()
            rec.append(([t.clone() for t in algo._flat], st))
        assert (algo._ro_graph is not None) == graph
        outs.append(rec)
        venv.close()
    for (fa, sa), (fb, sb) in zip(*outs):
        for a, b in zip(fa, fb):
            assert torch.equal(a, b)
        assert sa["episodes"] == sb["episodes"]
