"""Shared fixtures.  `gpu` marks tests that need an MI355X (run with -m gpu on the box)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def native():
    """The built C-ABI library (fails loudly if it is missing)."""
    from eraytracer_amd import _native as N
    N.lib()
    return N
