import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "unitree-rl-gym_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP simulator)")


@pytest.fixture(scope="session")
def oracle_lib():
    import bridge
    return bridge.ensure_built()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
