import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture
def gym():
    from isaacgym import gymapi
    return gymapi.acquire_gym()


def has_gpu():
    from test_isaacgym_amd import _native
    return _native.device_count() > 0
