"""Horovod variant of the cifar10 example (reference: examples/horovod_cifar10_resnet.py).

Horovod is not part of the MI355X stack this framework targets (no wheel in
the ROCm image, and the reference's HorovodBackend ignored process groups, so
HYBRID_OPT could not work on it: SURVEY.md section 2.2 B2).  Data parallelism
runs on torch.distributed with the `nccl` backend, which is RCCL over xGMI:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        examples/torch_cifar10_resnet.py <same flags>

This stub keeps the reference's file layout and exits with that instruction.
"""
import sys

MSG = ('Horovod is not supported by distributed_kfac_pytorch_amd; launch '
       'examples/torch_cifar10_resnet.py with torch.distributed.run (RCCL) instead.')

if __name__ == '__main__':
    print(MSG, file=sys.stderr)
    sys.exit(2)
