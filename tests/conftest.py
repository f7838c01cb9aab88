import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "faithdiff-dev_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU oracle case")


@pytest.fixture(autouse=True)
def _parity_current_test(request):
    """tests/golden/parity.py records every measured metric under the running test's id."""
    import parity
    parity.CURRENT["test"] = request.node.nodeid
    yield
    parity.CURRENT["test"] = None


def pytest_sessionfinish(session, exitstatus):
    import parity
    path = parity.dump()
    if path:
        print(f"\nparity metrics of {len(parity.RECORDS)} tests -> {path}")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"))
