"""Probe for the roofline table (profiles/README.md): one ResNet-50 K-FAC step
at batch 32 (bf16 autocast; grouped factor SYRK, fused eigensolver for all 108
factors, fused preconditioning chain), then 3 more fp32 and 3 bf16x3 chain runs.
Run under rocprofv3 --kernel-trace --stats (durations) and --pmc passes
(counters); kernels are matched by name."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402
from distributed_kfac_pytorch_amd.ops import precond_fused  # noqa: E402

dev = torch.device('cuda')
torch.manual_seed(0)
m = resnet.resnet50().to(dev).to(memory_format=torch.channels_last)
pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=1, lr=0.1, precond_precision='fp32',
                use_hip_graphs=False)
x = torch.randn(32, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev)
with torch.autocast('cuda', dtype=torch.bfloat16):
    loss = F.cross_entropy(m(x), y)
loss.backward()
pre.step()
torch.cuda.synchronize()
for _ in range(3):
    pre.fused.run(damping=1e-3)
bf = precond_fused.FusedPreconditioner(pre.fused.layers, 'bf16x3')
bf.refresh_eigen()
for _ in range(3):
    bf.run(damping=1e-3)
torch.cuda.synchronize()
print('ok', float(loss))
