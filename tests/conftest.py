import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ekuiper-vioneta_amd"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libekgpu.so on the device)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import ekoracle
    ekoracle.build()
    return ekoracle
