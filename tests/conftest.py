import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def hip_lib():
    """The built HIP library; on a GPU box a missing library is a failure."""
    from psrsigsim_amd import _lib
    _lib.check_build_hash()        # the binary under test was built from this tree
    return _lib.lib()
