import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def tfa():
    import tiflash_amd
    tiflash_amd.lib()  # fails loudly when the HIP library is missing
    return tiflash_amd


@pytest.fixture(scope="session")
def ctx(tfa):
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = tfa.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="session")
def dev():
    import torch
    return torch.device("cuda", 0)
