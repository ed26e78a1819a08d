import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_sessionstart(session):
    """Build libcallfs_rs.so (no-op when its content hash is current) before any test
    module imports callfs_amd, and the C oracle."""
    import __graft_entry__
    __graft_entry__.build()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def native_lib():
    """libcallfs_rs.so, built at session start."""
    from callfs_amd import _native
    return _native
