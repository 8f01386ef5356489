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


def _first_diff(a, b):
    return next((i for i, (x, y) in enumerate(zip(a, b)) if x != y), min(len(a), len(b)))


def pytest_assertrepr_compare(op, left, right):
    """Short reports for JPEG / plane byte comparisons: pytest's default diff of two 100 KB byte
    strings (or lists of them) runs for minutes and turns a mismatch into a test timeout."""
    if op != "==":
        return None
    if isinstance(left, (bytes, bytearray)) and isinstance(right, (bytes, bytearray)):
        return [f"bytes differ: {len(left)} vs {len(right)} B, first difference at offset {_first_diff(left, right)}"]
    if isinstance(left, (list, tuple)) and isinstance(right, (list, tuple)) and any(
            isinstance(v, (bytes, bytearray)) for v in list(left) + list(right)):
        bad = [i for i, (x, y) in enumerate(zip(left, right)) if x != y]
        return [f"sequences differ: lengths {len(left)} vs {len(right)}, unequal items {bad[:16]}"]
    return None


def golden(name: str) -> str:
    return os.path.join(GOLDEN, name)


def read(path: str) -> bytes:
    with open(path, "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def engine():
    import h2j
    return h2j.Engine()
