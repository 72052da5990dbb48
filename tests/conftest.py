import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU checks (still part of the default suite)")


@pytest.fixture(scope="session")
def rt():
    import rtref
    return rtref.package()


@pytest.fixture(scope="session")
def oracle():
    import rtref
    return rtref.Oracle()
