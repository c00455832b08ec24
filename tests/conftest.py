import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU-side test")


@pytest.fixture(scope="session")
def plays():
    import hgref
    return hgref.load_plays()


@pytest.fixture(scope="session")
def kat():
    import hgref
    return hgref.load_kat()
