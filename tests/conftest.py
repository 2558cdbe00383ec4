import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def golden6():
    return dict(np.load(os.path.join(GOLDEN, "rocket6dof_ref.npz")))


@pytest.fixture(scope="session")
def golden3():
    return dict(np.load(os.path.join(GOLDEN, "rocket3dof_ref.npz")))


@pytest.fixture(scope="session")
def golden6_x():
    return dict(np.load(os.path.join(GOLDEN, "rocket6dof_ref_xstack.npz")))


@pytest.fixture(scope="session")
def golden3_x():
    return dict(np.load(os.path.join(GOLDEN, "rocket3dof_ref_xstack.npz")))


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.load()
    return oracle
