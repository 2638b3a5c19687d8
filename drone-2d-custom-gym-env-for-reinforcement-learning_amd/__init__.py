"""MI355X-native batched Drone2dEnv (drop-in for the reference's ``Drone2dEnv.step`` hot path).

Import as ``drone2d_amd`` (the top-level ``drone2d_amd.py`` loader maps the package directory,
whose name is not a Python identifier, to that module name).

    import drone2d_amd as d2
    from drone2d_amd.config import ENV_TRAIN_CONFIG
    venv = d2.Drone2dVecEnv(65536, **dict(ENV_TRAIN_CONFIG, scenario="corridor"))
    obs = venv.reset(seed=0)
    obs, rew, term, trunc, info = venv.step(torch.rand(65536, 2, device="cuda") * 2 - 1)
"""
from . import abi, config, scenarios  # noqa: F401  (pure-Python, no GPU needed)

__all__ = ["abi", "config", "scenarios", "Drone2dVecEnv", "Drone2dEnv", "lib_path"]


def lib_path() -> str:
    from ._native import LIB_PATH

    return LIB_PATH


def __getattr__(name):
    # the env classes import torch + load libdrone2d_hip.so; defer until asked for
    if name in ("Drone2dVecEnv", "Drone2dEnv", "info_dicts"):
        from . import env

        return getattr(env, name)
    if name in ("SB3VecEnv",):
        from . import sb3

        return getattr(sb3, name)
    raise AttributeError(name)
