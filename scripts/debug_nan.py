"""Debug: where does the first non-finite value appear when graph replays follow
an eager inverse step with zero_grad(set_to_none=True)?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd import graphs
from distributed_kfac_pytorch_amd.models import resnet

dev = torch.device('cuda:0')
torch.manual_seed(0)
torch.backends.cudnn.benchmark = True
model = resnet.resnet50().to(dev).to(memory_format=torch.channels_last)
opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5)
pre = kfac.KFAC(model, damping=0.001, factor_update_freq=10, inv_update_freq=100, kl_clip=0.001,
                lr=0.0125, distribute_layer_factors=False, precond_precision='bf16x3')
x = torch.randn(32, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev)
STN = bool(int(os.environ.get('STN', '1')))

def train_step():
    opt.zero_grad(set_to_none=STN)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        loss = F.cross_entropy(model(x), y, label_smoothing=0.1)
    loss.backward()
    pre.step()
    opt.step()
    return loss

step = graphs.GraphedTrainStep(train_step, pre, [opt], enabled=True)
for _ in range(10):
    step()
step.prepare()
pre.param_groups[0]['step'] = 0

def finite(t):
    return bool(torch.isfinite(t).all().item())

def report(tag):
    torch.cuda.synchronize()
    bad = []
    if not all(finite(p) for p in model.parameters()): bad.append('params')
    if not all(finite(b) for b in model.buffers() if b.is_floating_point()): bad.append('buffers')
    if pre.plan is not None:
        if not finite(pre.plan.grad_arena): bad.append('pgrad_arena')
        if pre.plan.eig_arena is not None and not finite(pre.plan.eig_arena): bad.append('eig_arena')
    f = pre.fused
    if f is not None:
        for b in f.bufs:
            for name in ('QA', 'QG', 'QAt', 'QGt', 'Gct', 'T1', 'T2t', 'T3'):
                if not finite(getattr(b, name).t.float()):
                    bad.append('%s:%s' % (name, b.layer.module.__class__.__name__)); break
        if not finite(f.kl): bad.append('kl')
    for l in pre.layers:
        if not finite(l.state['A'].float()) or not finite(l.state['G'].float()):
            bad.append('factors'); break
    mom = [s.get('momentum_buffer') for s in opt.state.values()]
    if not all(m is None or finite(m) for m in mom): bad.append('momentum')
    print(tag, 'step=%d' % pre.param_groups[0]['step'], 'non-finite:', bad or 'none', flush=True)

report('after prepare')
for i in range(4):
    loss = step()
    report('after timed step %d (loss %.4f)' % (i, float(loss.item())))
