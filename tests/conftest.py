import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "humanoid_mppi-rl_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libmppi_hip.so")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


def golden_sd(name, prefix=""):
    with np.load(os.path.join(GOLDEN, name)) as z:
        return {k[len(prefix):]: z[k] for k in z.files if k.startswith(prefix)}


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return True
