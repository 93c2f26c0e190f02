import os
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "decoupled-kg_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


@pytest.fixture(autouse=True)
def _double_default():
    # reference tests/modules/acquisition/conftest.py:9-12
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.double)
    yield
    torch.set_default_dtype(old)


@pytest.fixture(autouse=True)
def _seed():
    # reference tests/conftest.py:5-9
    state = torch.random.get_rng_state()
    torch.manual_seed(1234)
    yield
    torch.random.set_rng_state(state)
