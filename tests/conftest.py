import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden", "reference_golden.npz")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    return np.load(GOLDEN, allow_pickle=False)


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle as O

    O.lib()
    return O
