"""Multi-rank sharding on CPU (gloo, world size 2) -- SURVEY.md §8(e).

Each rank steps its contiguous block of a global batch (the C oracle stands in for the per-GPU
kernel: test infrastructure) with global env ids and the globally computed env -> scenario map;
the episode statistics are SUM-all-reduced through ``drone2d_amd.shard.allreduce_stats``.  The
gathered per-env outputs and the reduced statistics must equal one unsharded batch bit for bit.
The same helpers drive bench.py's RCCL path on GPUs.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_TOTAL = 301          # odd on purpose: uneven shards
STEPS = 60
SCN = ["corridor", "S_corridor", "large", "parallel", "perpendicular", "S_parallel", "impossible"]


def _kw():
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    return dict(ENV_TRAIN_CONFIG, scenario=SCN)


def _actions():
    return np.random.default_rng(11).uniform(-1, 1, (STEPS, N_TOTAL, 2)).astype(np.float32)


def _run(backend, acts):
    obs_all, rew_all = [], []
    backend.reset()
    for t in range(STEPS):
        obs, rew, term, trunc, info = backend.step(torch.from_numpy(acts[t]))
        obs_all.append(obs.clone())
        rew_all.append(rew.clone())
    return torch.stack(obs_all), torch.stack(rew_all), backend.episode_stats()


def _worker(rank, world, port, out_dir, hip=False):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import drone2d_amd  # noqa: F401
    from drone2d_amd import shard
    from oracle_backend import OracleVecBackend

    r, w, _ = shard.init_process_group_from_env("gloo")
    assert (r, w) == (rank, world)
    off, cnt = shard.shard_range(N_TOTAL, world, rank)
    es = shard.shard_env_scenario(shard.global_env_scenario(N_TOTAL, len(SCN)), off, cnt)
    if hip:  # this rank's HIP shard (every rank on cuda:0 of a one-GPU box; gloo for the gathers)
        be = shard.make_shard_venv(N_TOTAL, rank, world, device=torch.device("cuda", 0), seed=21, **_kw())
        assert be.cfg.env_id_base == off and np.array_equal(be.env_scenario, es)
    else:
        be = OracleVecBackend(cnt, seed=21, env_scenario=es, env_id_offset=off, **_kw())
    obs, rew, stats = _run(be, _actions()[:, off:off + cnt])
    obs, rew = obs.cpu(), rew.cpu()
    stats = shard.allreduce_stats(stats.clone().cpu())
    # gather the per-env outputs (uneven shards: pad to the largest block)
    big = shard.shard_range(N_TOTAL, world, 0)[1]
    pad_o = torch.zeros(STEPS, big, 27)
    pad_o[:, :cnt] = obs
    pad_r = torch.zeros(STEPS, big)
    pad_r[:, :cnt] = rew
    go = [torch.zeros_like(pad_o) for _ in range(world)]
    gr = [torch.zeros_like(pad_r) for _ in range(world)]
    dist.all_gather(go, pad_o)
    dist.all_gather(gr, pad_r)
    if rank == 0:
        cnts = [shard.shard_range(N_TOTAL, world, k)[1] for k in range(world)]
        obs_g = torch.cat([g[:, :c] for g, c in zip(go, cnts)], 1)
        rew_g = torch.cat([g[:, :c] for g, c in zip(gr, cnts)], 1)
        torch.save({"obs": obs_g, "rew": rew_g, "stats": stats}, os.path.join(out_dir, "sharded.pt"))
    dist.barrier()
    dist.destroy_process_group()
    be.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    from drone2d_amd.shard import shard_range

    for n, w in ((65536, 8), (301, 2), (10, 3), (7, 7)):
        parts = [shard_range(n, w, r) for r in range(w)]
        assert parts[0][0] == 0 and sum(c for _, c in parts) == n
        for (o0, c0), (o1, _) in zip(parts, parts[1:]):
            assert o0 + c0 == o1
        assert max(c for _, c in parts) - min(c for _, c in parts) <= 1
    with pytest.raises(ValueError):
        shard_range(3, 4, 0)


def _sharded(tmp_path, hip):
    world = 2
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), hip)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return torch.load(os.path.join(tmp_path, "sharded.pt"), weights_only=True)


def test_two_rank_gloo_sharding_matches_single_batch(tmp_path, d2):
    from oracle_backend import OracleVecBackend

    got = _sharded(tmp_path, hip=False)
    single = OracleVecBackend(N_TOTAL, seed=21, **_kw())
    obs, rew, stats = _run(single, _actions())
    single.close()
    _check(got, obs, rew, stats)


@pytest.mark.gpu
def test_two_process_hip_shards_match_single_batch(tmp_path, d2):
    """Two processes, each stepping its HIP shard (env_id_offset, sliced scenario map) through
    libdrone2d_hip.so, gathered over gloo: identical to one unsharded HIP batch, bit for bit."""
    got = _sharded(tmp_path, hip=True)
    single = d2.Drone2dVecEnv(N_TOTAL, device=torch.device("cuda", 0), seed=21, **_kw())
    obs, rew, stats = _run(single, _actions())
    single.close()
    _check(got, obs.cpu(), rew.cpu(), stats.cpu())


def _check(got, obs, rew, stats):
    assert torch.equal(got["obs"], obs)
    assert torch.equal(got["rew"], rew)
    # per-env accumulators are identical; the reduction order differs (block sums), so compare the
    # integer counts exactly and the float sums to rounding
    np.testing.assert_array_equal(got["stats"][[1, 2, 3, 4]].numpy(), stats[[1, 2, 3, 4]].numpy())
    np.testing.assert_allclose(got["stats"].numpy(), stats.numpy(), rtol=1e-12, atol=1e-9)
    assert stats[1] > 0  # episodes finished


def _ppo_worker(rank, world, port, out_dir, hip=False):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import drone2d_amd  # noqa: F401
    from drone2d_amd import shard
    from drone2d_amd.ppo import PPO, PPOConfig
    from oracle_backend import OracleVecBackend

    shard.init_process_group_from_env("gloo")
    if hip:  # each rank's HIP shard on cuda:0 of the one-GPU box; gradients all-reduced over gloo
        off, cnt = shard.shard_range(4096, world, rank)
        be = shard.make_shard_venv(4096, rank, world, device=torch.device("cuda", 0), seed=5,
                                   **dict(_kw(), scenario="corridor"))
        cfg = PPOConfig.gpu_defaults(n_steps=8, batch_size=4096, n_epochs=2)
        algo = PPO(be, cfg, seed=rank)
        assert algo.manual is not None and algo.manual.lib is not None and not algo.use_graph
    else:
        off, cnt = shard.shard_range(64, world, rank)
        be = OracleVecBackend(cnt, seed=5, env_id_offset=off, **dict(_kw(), scenario="corridor"))
        # rank-dependent init seed on purpose: PPO broadcasts rank 0's parameters
        algo = PPO(be, PPOConfig(n_steps=8, batch_size=64, n_epochs=2), seed=rank, device="cpu")
    hist = algo.learn(2 * 8 * cnt)
    assert len(hist) == 2 and all(np.isfinite(h["value_loss"]) for h in hist)
    flat = torch.cat([p.detach().reshape(-1) for p in algo.policy.parameters()]).cpu()
    torch.save(flat, os.path.join(out_dir, f"ppo_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()
    be.close()


def _two_rank_ppo(tmp_path, hip):
    world = 2
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_ppo_worker, args=(r, world, port, str(tmp_path), hip)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    a = torch.load(os.path.join(tmp_path, "ppo_0.pt"), weights_only=True)
    b = torch.load(os.path.join(tmp_path, "ppo_1.pt"), weights_only=True)
    assert torch.equal(a, b)


def test_two_rank_ppo_keeps_one_policy(tmp_path, d2):
    """Data-parallel PPO over gloo: each rank rolls out its own env shard, gradients are averaged
    over the ranks every minibatch, so after two updates both ranks hold the same parameters."""
    _two_rank_ppo(tmp_path, hip=False)


@pytest.mark.gpu
def test_two_rank_ppo_hip_keeps_one_policy(tmp_path, d2):
    """The same with each rank's HIP env shard and the libd2d_ppo.so update kernels (two processes
    on the one GPU; the flat gradient buffer all-reduced over gloo before clip + Adam)."""
    _two_rank_ppo(tmp_path, hip=True)


_RCCL_SCRIPT = r'''
import os, sys
sys.path.insert(0, os.environ["D2D_REPO"])
import torch
import torch.distributed as dist
import drone2d_amd  # noqa: F401
from drone2d_amd import shard
from drone2d_amd.config import ENV_TRAIN_CONFIG

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
venv = shard.make_shard_venv(4096, 0, 1, seed=3, with_info=False, **dict(ENV_TRAIN_CONFIG, scenario="corridor"))
venv.reset()
for _ in range(120):
    venv.step(torch.rand(4096, 2, device="cuda") * 2 - 1)
stats = venv.episode_stats(clear=False).clone()
before = stats.clone()
dist.all_reduce(stats, op=dist.ReduceOp.SUM)   # the bench's one collective, on RCCL
torch.cuda.synchronize()
assert torch.equal(stats, before) and before[1].item() > 0, (stats, before)
venv.close()
dist.destroy_process_group()
print("RCCL_OK", int(before[1].item()))
'''


@pytest.mark.gpu
def test_rccl_backend_runs_the_stats_allreduce():
    """The `nccl` (RCCL) branch of the multi-GPU path on hardware: one rank (RCCL refuses two ranks on
    one device, and the 8-GPU runs are the driver's) initialises the RCCL process group the way
    ``shard.init_process_group_from_env`` does and all-reduces a real batch's episode-statistics
    vector on the device -- the fp64 SUM ``bench.py`` runs over ranks.  With one rank the sum is the
    vector itself, bit for bit."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", D2D_REPO=repo)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", _RCCL_SCRIPT], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
