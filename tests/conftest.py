import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

CONFIGS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the native extension")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def configs_dir():
    return CONFIGS
