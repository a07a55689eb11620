import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: full-size (BASELINE-scale) property checks")


@pytest.fixture(scope="session")
def mlls():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "mlls.npz")))


@pytest.fixture(scope="session")
def edge_cases():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "edge_cases.npz")))
