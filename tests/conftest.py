import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libgmcmc.so")
    config.addinivalue_line("markers", "slow: longer statistical tests")


@pytest.fixture(scope="session")
def oracle():
    from tests import _oracle
    return _oracle.load()


@pytest.fixture(scope="session")
def gm():
    """The product package with its HIP library; fails loudly when missing."""
    import general_mcmc_amd as g
    g._lib.require_gpu()
    return g
