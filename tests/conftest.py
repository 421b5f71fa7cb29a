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


@pytest.fixture(scope="session", autouse=True)
def _heartbeat():
    """Full-size oracle runs take minutes of silent CPU work: print a line every 60 s so a watchdog that
    kills silent runs can tell a long test from a hung one."""
    import threading
    import time
    stop = threading.Event()
    t0 = time.time()

    def beat():
        while not stop.wait(60):
            sys.__stderr__.write(f"[heartbeat] {time.time() - t0:.0f} s\n")
            sys.__stderr__.flush()
    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
