import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def tz():
    import tenzing_amd

    return tenzing_amd


@pytest.fixture(scope="session")
def gpu(tz):
    if tz.hip_device_count() == 0:
        pytest.fail("GPU test selected but no HIP device is visible")
    return 0
