"""Process-group bootstrap and DDP wrapping (one process per GPU).

`init_distributed()` reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* (set by
torch.distributed.run), binds the process to its GPU and initialises the
`nccl` backend (RCCL over xGMI on MI355X) or gloo on CPU; then selects the
K-FAC communication backend.  `wrap_ddp` builds the data-parallel gradient
all-reduce with bucket views so K-FAC can rewrite `.grad` in
place.  Reference launch path: examples/torch_imagenet_resnet.py:118-152
(which used device_ids=[local_rank] even on CPU, where it raises).
"""
import datetime
import os

import torch
import torch.distributed as dist

from .. import comm

__all__ = ['init_distributed', 'wrap_ddp', 'get_local_device', 'is_distributed']


def is_distributed():
    return int(os.environ.get('WORLD_SIZE', '1')) > 1


def get_local_device(no_cuda=False):
    if torch.cuda.is_available() and not no_cuda:
        # modulo the visible devices: a multi-rank rehearsal on a one-GPU box
        # (KFAC_DIST_BACKEND=gloo) puts every rank on cuda:0; on a full node
        # LOCAL_RANK < device_count and this is the identity
        n = max(1, torch.cuda.device_count())
        return torch.device('cuda', int(os.environ.get('LOCAL_RANK', '0')) % n)
    return torch.device('cpu')


def init_distributed(backend=None, no_cuda=False, timeout_s=1800):
    """Initialise torch.distributed when WORLD_SIZE > 1; returns the device."""
    device = get_local_device(no_cuda)
    if device.type == 'cuda':
        torch.cuda.set_device(device)
    if is_distributed() and not dist.is_initialized():
        if backend is None:
            # KFAC_DIST_BACKEND=gloo rehearses the multi-rank GPU path with
            # several ranks sharing one GPU (RCCL refuses duplicate devices)
            backend = os.environ.get('KFAC_DIST_BACKEND') or \
                ('nccl' if device.type == 'cuda' else 'gloo')
        kw = {}
        if backend == 'nccl' and device.type == 'cuda':
            kw['device_id'] = device
        dist.init_process_group(backend=backend, init_method='env://',
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    comm.reset_comm_backend()
    comm.init_comm_backend()
    return device


def wrap_ddp(model, device, bucket_cap_mb=None, broadcast_buffers=True):
    """DistributedDataParallel with gradient bucket views (single process: no-op)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return model
    kw = dict(gradient_as_bucket_view=True, broadcast_buffers=broadcast_buffers)
    if bucket_cap_mb is not None:
        kw['bucket_cap_mb'] = bucket_cap_mb
    if device.type == 'cuda':
        return torch.nn.parallel.DistributedDataParallel(model, device_ids=[device.index], **kw)
    return torch.nn.parallel.DistributedDataParallel(model, **kw)
