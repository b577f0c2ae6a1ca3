import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built HIP kernels")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    """Skip-free GPU fixture: `-m gpu` tests must FAIL (not skip) when the native path is absent."""
    import torch

    assert torch.cuda.is_available(), "gpu test collected but no GPU is visible"
    from llm_weighted_consensus_amd import ops

    ops.kernels()  # raises loudly if _kernels.so is missing
    return torch.device("cuda:0")
