import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "h264-h265-to-jpeg_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def golden(name: str) -> str:
    return os.path.join(GOLDEN, name)


def read(path: str) -> bytes:
    with open(path, "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def engine():
    import h2j
    return h2j.Engine()
