import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (run with -m gpu on an MI355X)")
    config.addinivalue_line("markers", "ref: needs /root/reference (the reference source tree)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def mh():
    import metalhuffman_amd.build as B
    B.build()
    import metalhuffman_amd
    return metalhuffman_amd


@pytest.fixture(scope="session")
def bigbridge():
    from metalhuffman_amd import frames
    return frames.bigbridge()


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a HIP device")
    return torch.device("cuda:0")


def rng(seed=0):
    return np.random.default_rng(seed)
