"""Test infrastructure: the C oracle presented with Drone2dVecEnv's interface (torch CPU tensors),
so host-side layers (the SB3 adapter, sharding) can be exercised without a GPU.  Never shipped."""
import numpy as np
import torch


class OracleVecBackend:
    def __init__(self, num_envs, seed=0, env_scenario=None, timeup_truncates=False, env_id_offset=0,
                 envs_total=None, exact_trig=False, **kwargs):
        import oracle

        import drone2d_amd  # noqa: F401
        from drone2d_amd.config import make_cfg
        from drone2d_amd.env import _make_box, build_scenarios, is_curriculum, is_fresh_curriculum, make_curriculum

        oracle.build()
        self.kwargs = dict(kwargs)
        self.num_envs = int(num_envs)
        fresh = is_fresh_curriculum(self.kwargs)
        self.scenarios = [] if fresh else build_scenarios(self.kwargs)
        if env_scenario is None:
            env_scenario = 2 * np.arange(self.num_envs) if fresh else np.arange(self.num_envs) % len(self.scenarios)
        self.env_scenario = np.ascontiguousarray(np.asarray(env_scenario, dtype=np.int32))
        self.cfg = make_cfg(dict(self.kwargs), auto_reset=True, timeup_truncates=timeup_truncates,
                            env_id_base=env_id_offset)
        # as Drone2dVecEnv: fresh curriculum (2), curriculum pool (1), test scenarios (0)
        self.cfg.scn_pool = (2 if fresh else 1) if is_curriculum(self.kwargs) else 0
        cur = make_curriculum(self.kwargs, envs_total or self.num_envs) if fresh else None
        self.orc = oracle.OracleBatch(self.cfg, [s.to_c() for s in self.scenarios], self.num_envs,
                                      env_scenario=self.env_scenario, curriculum=cur, exact_trig=exact_trig)
        self.seed_value = int(seed)
        self.action_space = _make_box(-np.ones(2), np.ones(2))
        self.observation_space = _make_box(-np.ones(27), np.ones(27))
        self.device = torch.device("cpu")

    def reset(self, seed=None, mask=None):
        if seed is not None:
            self.seed_value = int(seed)
        return torch.from_numpy(self.orc.reset(self.seed_value, mask))

    def step(self, actions):
        a = actions.cpu().numpy() if isinstance(actions, torch.Tensor) else np.asarray(actions, np.float32)
        obs, rew, term, trunc, info = self.orc.step(a)
        return (torch.from_numpy(obs), torch.from_numpy(rew), torch.from_numpy(term), torch.from_numpy(trunc),
                torch.from_numpy(info))

    @property
    def terminal_obs(self):
        return torch.from_numpy(self.orc.tobs.copy())

    def episode_stats(self, clear=True):
        return torch.from_numpy(self.orc.episode_stats(clear))

    def close(self):
        self.orc.close()
