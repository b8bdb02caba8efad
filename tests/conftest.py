import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP) device')
    config.addinivalue_line('markers', 'slow: long-running test')


@pytest.fixture(autouse=True)
def _reset_comm():
    from distributed_kfac_pytorch_amd import comm
    comm.reset_comm_backend()
    yield
    comm.reset_comm_backend()


def gpu_available():
    import torch
    return torch.cuda.is_available()
