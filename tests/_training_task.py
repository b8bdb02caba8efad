"""A small learnable CIFAR-shaped task for the multi-step training-quality
checks: ResNet-20 (models/resnet_cifar.py) on smooth
class templates plus noise, SGD + K-FAC with factors every step and inverses every
10 steps, 100 steps.  The reference K-FAC's loss curve on it is the fixture
tests/fixtures/training_quality_resnet20.pt (scripts/make_training_fixture.py,
which runs the READ-ONLY reference in a subprocess); this framework's CPU path
must reproduce it, its GPU fp32 path track it, and the bench configuration stay
within a band of the GPU fp32 run (tests/test_training_quality.py,
tests/test_gpu_training_quality.py).

Reference training loop: examples/torch_cifar10_resnet.py:110-194 and
examples/cnn_utils/engine.py:9-93 (forward, loss, backward, preconditioner
step, optimizer step).
"""
import torch
import torch.nn.functional as F

STEPS = 100
BATCH = 32
CLASSES = 10
SNR = 0.2             # template scale against unit noise
LR = 0.05
KFAC_KW = dict(lr=LR, factor_decay=0.95, damping=0.003, kl_clip=0.001,
               factor_update_freq=1, inv_update_freq=10)
SGD_KW = dict(lr=LR, momentum=0.9, weight_decay=5e-4)
FIXTURE = 'tests/fixtures/training_quality_resnet20.pt'


def batches(steps=STEPS, batch=BATCH):
    """The task's batches (CPU, fixed seed): x = SNR * template[y] + noise,
    templates smooth (bilinear 4x4 -> 32x32) so convolutions can see them."""
    g = torch.Generator().manual_seed(2024)
    templates = F.interpolate(torch.randn(CLASSES, 3, 4, 4, generator=g), size=32,
                              mode='bilinear', align_corners=False)
    out = []
    for _ in range(steps):
        y = torch.randint(0, CLASSES, (batch,), generator=g)
        x = SNR * templates[y] + torch.randn(batch, 3, 32, 32, generator=g)
        out.append((x, y))
    return out


def model():
    from distributed_kfac_pytorch_amd.models import resnet_cifar
    torch.manual_seed(0)
    return resnet_cifar.resnet20()


def loss_fn(out, y):
    return F.cross_entropy(out, y)


def run_eager(net, pre, data, device='cpu'):
    """Plain eager loop (the reference's engine order); returns per-step losses."""
    opt = torch.optim.SGD(net.parameters(), **SGD_KW)
    losses = []
    for x, y in data:
        x, y = x.to(device), y.to(device)
        opt.zero_grad()
        loss = loss_fn(net(x), y)
        loss.backward()
        if pre is not None:
            pre.step()
        opt.step()
        losses.append(float(loss.detach()))
    return losses


def window_means(losses, width=25):
    return [sum(losses[i:i + width]) / len(losses[i:i + width])
            for i in range(0, len(losses), width)]
