"""Stage-by-stage ResNet-50 K-FAC step on cuda:0 with faulthandler (debug aid)."""
import faulthandler
import os
import sys
import time

faulthandler.enable(all_threads=True)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.models import resnet

solver = sys.argv[1] if len(sys.argv) > 1 else 'auto'
graphs = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = torch.device('cuda:0')
torch.manual_seed(0)
model = resnet.resnet50().to(dev).to(memory_format=torch.channels_last)
opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9)
pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=1, lr=0.01, eigen_solver=solver,
                use_hip_graphs=bool(graphs))
x = torch.randn(32, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev)
for it in range(3):
    t0 = time.time()
    with torch.autocast('cuda', dtype=torch.bfloat16):
        loss = F.cross_entropy(model(x), y)
    loss.backward()
    torch.cuda.synchronize(); print('fwd/bwd ok', flush=True)
    p = pre.param_groups[0]
    pre.compute_factors(alpha=p['factor_decay']); torch.cuda.synchronize(); print('factors ok', flush=True)
    pre.allreduce_factors()
    if not pre.workers_assigned:
        pre._assign_workers(); pre.workers_assigned = True
    print('assigned', flush=True)
    pre.compute_inverses(damping=p['damping']); torch.cuda.synchronize(); print('inverses ok', flush=True)
    pre.compute_preconditioned_gradients(damping=p['damping']); torch.cuda.synchronize(); print('precond ok', flush=True)
    s = pre._compute_grad_scale(); pre.update_gradients(s); torch.cuda.synchronize(); print('update ok', flush=True)
    p['step'] += 1
    opt.step(); opt.zero_grad()
    torch.cuda.synchronize()
    print('iter', it, 'loss', loss.item(), 'time', time.time() - t0, flush=True)
print('debug smoke ok', solver)
