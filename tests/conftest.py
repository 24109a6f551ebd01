import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


# The hot-path parity files run first, so that `pytest -x` cannot hide the rasterizer's results behind an unrelated
# early failure (the default order is alphabetical).
FIRST = ("test_gpu_raster.py", "test_gpu_fullsize.py", "test_gpu_aux.py", "test_gpu_boundary.py")


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return FIRST.index(name) if name in FIRST else len(FIRST)
    items.sort(key=rank)   # stable: the order inside each file is kept


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def hip_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from dogs_amd import build as B
    B.build()
    return torch.device("cuda:0")
