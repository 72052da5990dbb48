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
    # On a GPU box torch must initialise its HIP runtime before librt_hw_amd.so is loaded
    # (see test_gpu_parity.py), also when CPU tests that load the library run first.
    try:
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")
    except ImportError:
        pass
    import rtref
    return rtref.package()


@pytest.fixture(scope="session")
def oracle():
    import rtref
    return rtref.Oracle()
