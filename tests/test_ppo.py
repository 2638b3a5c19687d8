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
    """The HIP-graph replayed update (shuffles + every minibatch step) computes what the eager update
    computes (bs = 12288: every epoch ends with a ragged 8 192-sample minibatch)."""
    from drone2d_amd.ppo import PPO, PPOConfig

    params = []
    for graph in (False, True):
        venv = d2.Drone2dVecEnv(4096, seed=1, **_kw(scenario="corridor"))
        cfg = PPOConfig.gpu_defaults(n_steps=8, batch_size=bs, n_epochs=4 if bs > 4096 else 2)
        cfg.graph = graph
        algo = PPO(venv, cfg, seed=0)
        assert algo.use_graph == graph
        hist = algo.learn(3 * 8 * 4096)  # the first update runs eagerly, the next two replay the graph
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
@pytest.mark.parametrize("scn", ["corridor", "fresh_curriculum"])
def test_rollout_graph_matches_eager(d2, scn):
    """The captured rollout (policy + env step + GAE replayed as one HIP graph) fills the same
    buffers as the eager loop, bit for bit, over five consecutive rollouts (the first eager, the
    second captured and replayed, then three more replays).  ``fresh_curriculum`` is the
    configuration of profiles/r04/ppo/crash_fresh_graph_memset.err (an illegal address at the second
    rollout-graph replay): the device scenario generator K5 and K1's FreshRing
    appends inside PPO's rollout graph with the policy kernels between the steps; stage 4 -> 5 of
    the schedule during the rollouts."""
    from drone2d_amd.ppo import PPO, PPOConfig

    kw = _kw(scenario="corridor") if scn == "corridor" else _kw(mode="curriculum", scenario="curriculum",
                                                                 sim_num=1990000)
    outs = []
    for graph in (False, True):
        venv = d2.Drone2dVecEnv(2048, seed=4, with_info=True, **kw)
        assert venv.fresh == (scn != "corridor")
        cfg = PPOConfig.gpu_defaults(n_steps=16, batch_size=4096)
        cfg.graph = graph
        algo = PPO(venv, cfg, seed=2)
        rec = []
        for _ in range(5):
            st = algo.collect_rollouts()
            rec.append(([t.clone() for t in algo._flat], st))
        assert (algo._ro_graph is not None) == graph
        if venv.fresh:
            rec.append(([torch.as_tensor(np.frombuffer(bytes(venv.scenario_table()), np.uint8))], {"episodes": 0}))
        outs.append(rec)
        venv.close()
    for (fa, sa), (fb, sb) in zip(*outs):
        for a, b in zip(fa, fb):
            assert torch.equal(a, b)
        assert sa["episodes"] == sb["episodes"]
    assert sum(s["episodes"] for _, s in outs[1]) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 5, 1000, 32775, 1 << 20])
def test_permute_gives_permutations(d2, n):
    """d2d_ppo_permute: every epoch's row is a permutation of [0, n), the epochs differ, and the
    device counter advances so the next call (a graph replay) draws new shuffles."""
    from drone2d_amd.ppo import ppo_native

    lib = ppo_native()
    E = 3
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = torch.empty(E * n, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    assert lib.d2d_ppo_permute(n, E, 12345, ctr.data_ptr(), out.data_ptr(), st) == 0
    first = out.clone()
    assert lib.d2d_ppo_permute(n, E, 12345, ctr.data_ptr(), out.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert int(ctr) == 2 * E
    ar = torch.arange(n, device="cuda")
    for rows in (first, out):
        for e in range(E):
            assert torch.equal(torch.sort(rows[e * n:(e + 1) * n]).values, ar)
    if n >= 1000:
        assert not torch.equal(first[:n], first[n:2 * n]) and not torch.equal(first, out)
        # a shuffle, not a shift: the first half of a permutation holds about half of every residue
        lo = first[:n // 2]
        assert abs(float((lo < n // 2).float().mean()) - 0.5) < 0.06


def _torch_policy_step(pol, obs, noise):
    with torch.no_grad():
        mean, value = pol(obs)
        act = mean + pol.log_std.exp() * noise
        return act, pol.log_prob(mean, act), value


@pytest.mark.gpu
@pytest.mark.parametrize("n", [37, 4096, 65536 + 100])
def test_rollout_step_matches_torch(d2, n):
    """d2d_ppo_rollout_step against the torch restatement (ppo.py _rollout_body, compute_gae): step
    0's actions / log-densities / values / clipped env actions / observation copy, step t's record
    of step t-1's rewards, dones and episode statistics, and step T's bootstrap value + GAE (bit for
    bit where the bootstrap value drops out, to the MLP's float tolerance where it enters)."""
    import ctypes as C

    from drone2d_amd import abi
    from drone2d_amd.ppo import ActorCritic, D2DPPORollout, ManualStep, PPOConfig, compute_gae

    torch.manual_seed(0)
    pol = ActorCritic()
    with torch.no_grad():
        pol.log_std.copy_(torch.tensor([-0.4, 0.3]))
        pol.action_net.weight.mul_(60.0)  # actions beyond [-1, 1]: the clip is exercised
    pol = pol.cuda()
    man = ManualStep(pol, PPOConfig(), "cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    T = 4
    obs = torch.rand(n, 27, device="cuda", generator=g) * 2 - 1
    noise = torch.randn(T, n, 2, device="cuda", generator=g)
    f = lambda *sh, dt=torch.float32: torch.full(sh, float("nan"), device="cuda").to(dt)  # noqa: E731
    obs_buf, act_buf, logp_buf, val_buf, rew_buf = f(T, n, 27), f(T, n, 2), f(T, n), f(T, n), f(T, n)
    adv_buf, ret_buf, act_env = f(T, n), f(T, n), f(n, 2)
    done_buf = torch.zeros(T, n, dtype=torch.bool, device="cuda")
    start0 = torch.ones(n, dtype=torch.bool, device="cuda")
    stats = torch.zeros(T, (n + 63) // 64, 2, dtype=torch.float64, device="cuda")
    ptr = lambda x: x.data_ptr() if x is not None else None  # noqa: E731
    cfg = PPOConfig()
    r = D2DPPORollout(n=n, T=T, info_dim=abi.INFO_DIM, info_totrew=abi.INFO_TOTREW, gamma=cfg.gamma,
                      gae_lambda_gamma=cfg.gamma * cfg.gae_lambda, log_std=ptr(pol.log_std), obs_buf=ptr(obs_buf),
                      act_buf=ptr(act_buf), logp_buf=ptr(logp_buf), val_buf=ptr(val_buf), rew_buf=ptr(rew_buf),
                      done_buf=ptr(done_buf), start0=ptr(start0), act_env=ptr(act_env), adv_buf=ptr(adv_buf),
                      ret_buf=ptr(ret_buf), stats=ptr(stats))
    st = torch.cuda.current_stream().cuda_stream
    lib = man.lib
    # step 0 (no previous step)
    r.t, r.obs, r.noise = 0, ptr(obs), ptr(noise[0])
    assert lib.d2d_ppo_rollout_step(C.byref(r), man.weight_ptrs(), st) == 0
    a_ref, lp_ref, v_ref = _torch_policy_step(pol, obs, noise[0])
    torch.cuda.synchronize()
    assert torch.equal(obs_buf[0], obs)
    torch.testing.assert_close(act_buf[0], a_ref, rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(logp_buf[0], lp_ref, rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(val_buf[0], v_ref, rtol=1e-5, atol=2e-5)
    assert torch.equal(act_env, act_buf[0].clamp(-1.0, 1.0))
    frac = float((act_buf[0].abs() > 1).float().mean())
    assert n < 1000 or 0.05 < frac < 0.95
    # steps 1 .. T-1: each records its predecessor's env outputs
    rews = torch.randn(T, n, device="cuda", generator=g)
    terms = torch.rand(T, n, device="cuda", generator=g) < 0.2
    truncs = torch.rand(T, n, device="cuda", generator=g) < 0.05
    info = torch.randn(T, n, abi.INFO_DIM, device="cuda", generator=g)
    for t in range(1, T + 1):
        o = obs if t < T else torch.rand(n, 27, device="cuda", generator=g)
        r.t, r.obs, r.noise = t, ptr(o), ptr(noise[t]) if t < T else None
        r.prev_rew, r.prev_term, r.prev_trunc, r.prev_info = (ptr(rews[t - 1]), ptr(terms[t - 1]),
                                                             ptr(truncs[t - 1]), ptr(info[t - 1]))
        assert lib.d2d_ppo_rollout_step(C.byref(r), man.weight_ptrs(), st) == 0
    torch.cuda.synchronize()
    dones = terms | truncs
    assert torch.equal(rew_buf, rews) and torch.equal(done_buf, dones)
    assert torch.equal(start0, dones[T - 1])
    ep = stats.sum(1)
    assert torch.equal(ep[:, 0], dones.sum(1).double())
    ret_ref = torch.where(dones, info[..., abi.INFO_TOTREW].double(), 0.0).sum(1)
    torch.testing.assert_close(ep[:, 1], ret_ref, rtol=1e-12, atol=1e-9)
    # GAE against compute_gae on the kernel's own values
    last_v = _torch_policy_step(pol, o, noise[0])[2]
    starts = torch.cat([torch.ones(1, n, dtype=torch.bool, device="cuda"), dones[:-1]])
    adv_ref, ret_ref = compute_gae(rew_buf, val_buf, starts, last_v, dones[T - 1], cfg.gamma, cfg.gae_lambda)
    torch.testing.assert_close(adv_buf, adv_ref, rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(ret_buf, ret_ref, rtol=1e-5, atol=2e-5)
    # where step T-1 ended the episode, the bootstrap value drops out: same bits as torch
    d = dones[T - 1]
    assert torch.equal(adv_buf[:, d], adv_ref[:, d]) and torch.equal(ret_buf[:, d], ret_ref[:, d])


@pytest.mark.gpu
@pytest.mark.parametrize("M", [64, 1000, 32768, 40000])
def test_fused_grad_matches_separate_kernels(d2, M):
    """d2d_ppo_fused_grad + d2d_ppo_grad_reduce (forward, head, backward and weight gradients in one
    launch, per-sample state on chip) against the separate forward / backward / wgrad kernels on
    the same minibatch: every gradient and the loss statistics agree up to summation order."""
    from drone2d_amd.ppo import ActorCritic, ManualStep, PPOConfig

    torch.manual_seed(11)
    base = ActorCritic()
    with torch.no_grad():
        base.log_std.copy_(torch.tensor([-0.3, 0.2]))
        base.action_net.weight.mul_(30.0)
    cfg = PPOConfig()
    g = torch.Generator().manual_seed(12)
    T = 50000
    rollout = tuple(t.cuda() for t in (torch.randn(T, 27, generator=g) * 0.5, torch.randn(T, 2, generator=g),
                                       torch.randn(T, generator=g) - 3.0, torch.randn(T, generator=g),
                                       torch.randn(T, generator=g) * 3))
    idx = torch.randperm(T, generator=g)[:M].cuda()
    out = []
    for fused in (False, True):
        pol = ActorCritic()
        pol.load_state_dict(base.state_dict())
        step = ManualStep(pol.cuda(), cfg, "cuda")
        step.fused = fused
        acc = {k: torch.zeros((), device="cuda") for k in ("policy_loss", "value_loss", "entropy", "clip_fraction")}
        with torch.no_grad():
            step.grad(idx, rollout, acc)
        torch.cuda.synchronize()
        out.append((step.G.clone(), {k: v.clone() for k, v in acc.items()},
                    [n for n, _ in pol.named_parameters()], [p.grad.numel() for p in pol.parameters()]))
    (ga, aa, names, sizes), (gb, ab, _, _) = out
    for name, a, b in zip(names, torch.split(ga, sizes), torch.split(gb, sizes)):
        torch.testing.assert_close(b, a, rtol=2e-4, atol=1e-6, msg=name)
    for k in aa:
        torch.testing.assert_close(ab[k], aa[k], rtol=1e-5, atol=1e-6, msg=k)
