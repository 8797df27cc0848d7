import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP decode path)")


@pytest.fixture(scope="session")
def gpu_ready():
    """Fail loudly (not skip) when a gpu-marked test runs without a working HIP path."""
    import zflac_amd

    n = zflac_amd.device_count()
    assert n > 0, "gpu test selected but no HIP device is visible"
    return n
