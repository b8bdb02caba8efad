"""Debug: the fused preconditioning chain eager vs hipGraph replay (ResNet-50)."""
import os
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, os.getcwd())
import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402

dev = torch.device('cuda')
torch.manual_seed(0)
model = resnet.get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=1, lr=0.0125, kl_clip=1e-3,
                distribute_layer_factors=False, precond_precision=os.environ.get('PREC', 'bf16x3'),
                use_hip_graphs=False)
x = torch.randn(32, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev)
with torch.autocast('cuda', dtype=torch.bfloat16):
    loss = F.cross_entropy(model(x), y)
loss.backward()
pre.step()
torch.cuda.synchronize()
f = pre.fused
# fresh gradients to precondition
model.zero_grad(set_to_none=False)
with torch.autocast('cuda', dtype=torch.bfloat16):
    loss = F.cross_entropy(model(x), y)
loss.backward()
torch.cuda.synchronize()
kl_e = f.run(damping=1e-3).clone()
pg_e = [l.pgrad_buffer.clone() for l in pre.layers]
torch.cuda.synchronize()
print('eager kl', float(kl_e), flush=True)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    f.run(damping=1e-3)   # warm-up on the capture stream
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    kl_ref = f.run(damping=1e-3)
for r in range(3):
    for l in pre.layers:
        l.pgrad_buffer.zero_()
    g.replay()
    torch.cuda.synchronize()
    err = max(float((l.pgrad_buffer - p).abs().max()) for l, p in zip(pre.layers, pg_e))
    print('replay', r, 'kl', float(f.kl), 'max |pgrad - eager|', err, flush=True)
