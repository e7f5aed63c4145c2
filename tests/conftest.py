import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        # a -m gpu run that cannot reach the HIP path must be red, not green-by-skip
        pytest.fail("no GPU visible: the -m gpu suite needs cuda:0 (MI355X)", pytrace=False)
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def ctx(cuda):
    from flashws_amd import gpu
    c = gpu.Ctx(0, max_frames=1 << 22, max_stream_bytes=1 << 30)
    yield c
    c.close()
