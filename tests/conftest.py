import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

SCENARIOS = ["perpendicular", "parallel", "S_parallel", "corridor", "S_corridor", "large", "impossible"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def golden_scn():
    return load_golden("scenarios")


@pytest.fixture(scope="session")
def golden_traj():
    return load_golden("traj")


@pytest.fixture(scope="session")
def golden_crafted():
    return load_golden("crafted")


@pytest.fixture(scope="session")
def golden_probe():
    return load_golden("path_probe")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # oracle/oracle.py

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def d2():
    import drone2d_amd

    return drone2d_amd


@pytest.fixture(scope="session")
def scenarios_c(d2):
    from drone2d_amd.scenarios import create_test_scenario

    return [create_test_scenario(s, 1300, 1300).to_c() for s in SCENARIOS]


@pytest.fixture(scope="session")
def ref_cfg(d2):
    from drone2d_amd.config import ENV_TRAIN_CONFIG, make_cfg

    return make_cfg(dict(ENV_TRAIN_CONFIG), auto_reset=False)


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
