"""RCCL at world size 1 (tests/_rccl_worker.py in a child process): the K-FAC
communication layer's collectives executed by a real RCCL communicator on the
GPU -- the factor arena all-reduce (fp32, bf16), the in-place arena
all-gather, broadcast, barrier -- and K-FAC steps with the 'nccl' process
group up.  Multi-rank RCCL needs more than the one GPU a test box has."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.skipif(not torch.cuda.is_available(), reason='needs a GPU')
def test_rccl_world_size_one_collectives():
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()),
               RANK='0', WORLD_SIZE='1', LOCAL_RANK='0')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tests', '_rccl_worker.py')],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=100)
    out = r.stdout + r.stderr
    print(out[-3000:])
    assert r.returncode == 0 and 'RCCL_W1_OK' in r.stdout, out[-3000:]
    assert 'all_reduce' in r.stdout and 'all_gather_into_tensor' in r.stdout
