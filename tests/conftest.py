"""Test configuration.

Markers: ``gpu`` = needs an MI355X (run on the GPU box with ``-m gpu``);
everything else runs on CPU.  The oracle (``oracle/``) is imported only by
tests, as the checker.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpc-mmd_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def native():
    from optimizer import _native
    if _native.lib().mpcmmd_device_count() < 1:
        raise RuntimeError("gpu test: no HIP device visible (these tests must run on the MI355X box)")
    return _native
