"""Datasets for the CNN examples (reference: examples/cnn_utils/datasets.py:1-68).

No network access and no torchvision on the target image, so:
  * CIFAR-10 is read from the *binary* distribution (`cifar-10-batches-bin/
    data_batch_{1..5}.bin`, `test_batch.bin`: 1 label byte + 3072 pixel bytes
    per record) when `--data-dir` holds it -- raw bytes, nothing unpickled;
  * otherwise (and always for ImageNet) a deterministic synthetic dataset of
    the right shapes is used: 3x32x32 / 10 classes, or 3x224x224 / 1000
    classes, normalised like the real data.
Every rank gets a DistributedSampler shard; the loader batch is
`batch_size * batches_per_allreduce` (micro-batched by the engine).
"""
import os

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import DataLoader, Dataset, TensorDataset
from torch.utils.data.distributed import DistributedSampler

__all__ = ['get_cifar', 'get_imagenet', 'make_sampler_and_loader', 'SyntheticImages']

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2023, 0.1994, 0.2010)


class SyntheticImages(Dataset):
    """Deterministic random images/labels (per-index generator)."""

    def __init__(self, n, shape, classes, seed=0):
        self.n, self.shape, self.classes, self.seed = n, shape, classes, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        x = torch.randn(self.shape, generator=g)
        y = int(torch.randint(0, self.classes, (1,), generator=g))
        return x, y


class _CifarBinary(Dataset):
    def __init__(self, files, train):
        raw = np.concatenate([np.fromfile(f, dtype=np.uint8).reshape(-1, 3073) for f in files])
        self.labels = torch.from_numpy(raw[:, 0].astype(np.int64))
        self.images = torch.from_numpy(raw[:, 1:].reshape(-1, 3, 32, 32).copy())
        self.train = train
        self.mean = torch.tensor(CIFAR_MEAN).view(3, 1, 1)
        self.std = torch.tensor(CIFAR_STD).view(3, 1, 1)

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        x = self.images[i].float() / 255.0
        if self.train:   # random crop (pad 4) + horizontal flip
            x = torch.nn.functional.pad(x, (4, 4, 4, 4))
            r, c = np.random.randint(0, 9, 2)
            x = x[:, r:r + 32, c:c + 32]
            if np.random.rand() < 0.5:
                x = x.flip(2)
        return (x - self.mean) / self.std, self.labels[i]


def get_cifar(args):
    d = os.path.join(args.data_dir, 'cifar-10-batches-bin') if args.data_dir else None
    if d and os.path.isdir(d):
        train = _CifarBinary([os.path.join(d, 'data_batch_%d.bin' % i) for i in range(1, 6)],
                             True)
        val = _CifarBinary([os.path.join(d, 'test_batch.bin')], False)
    else:
        n = getattr(args, 'synthetic_size', 50000)
        train = SyntheticImages(n, (3, 32, 32), 10, seed=1)
        val = SyntheticImages(max(n // 5, 1), (3, 32, 32), 10, seed=2)
    return (make_sampler_and_loader(args, train, shuffle=True),
            make_sampler_and_loader(args, val, shuffle=False, val=True))


def get_imagenet(args):
    n = getattr(args, 'synthetic_size', 1281167)
    size = getattr(args, 'image_size', 224)
    train = SyntheticImages(n, (3, size, size), 1000, seed=3)
    val = SyntheticImages(max(n // 25, 1), (3, size, size), 1000, seed=4)
    return (make_sampler_and_loader(args, train, shuffle=True),
            make_sampler_and_loader(args, val, shuffle=False, val=True))


def make_sampler_and_loader(args, dataset, shuffle=True, val=False):
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    sampler = DistributedSampler(dataset, num_replicas=world, rank=rank, shuffle=shuffle)
    bs = args.val_batch_size if val else args.batch_size * args.batches_per_allreduce
    loader = DataLoader(dataset, batch_size=bs, sampler=sampler,
                        num_workers=getattr(args, 'workers', 0),
                        pin_memory=getattr(args, 'cuda', False), drop_last=not val)
    return sampler, loader
