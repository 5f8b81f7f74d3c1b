import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblakeside_gpu.so on the device)")


@pytest.fixture(scope="session")
def engine():
    """One HIP engine for the whole GPU session (one process on the card)."""
    from lakeside_amd.evaluator import Engine
    e = Engine(0)
    yield e
    e.close()
