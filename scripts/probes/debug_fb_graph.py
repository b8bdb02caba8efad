"""Debug: graph-replayed forward/backward + eager K-FAC, with the gradients checked
between the replay and K-FAC (is the replayed backward or K-FAC at fault?)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.getcwd())
import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402

dev = torch.device('cuda')
torch.manual_seed(1234)
torch.backends.cudnn.benchmark = not os.environ.get('NOBENCH')
MF = torch.contiguous_format if os.environ.get('NCHW') else torch.channels_last
model = resnet.get_model(os.environ.get('MODEL', 'resnet50')).to(dev).to(
    memory_format=MF)
opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5)
use_kfac = not os.environ.get('NOKFAC')
pre = kfac.KFAC(model, damping=1e-3, factor_update_freq=1000, inv_update_freq=1000, kl_clip=1e-3,
                lr=0.0125, distribute_layer_factors=False, precond_precision='bf16x3',
                use_hip_graphs=False) if use_kfac else None
g0 = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(32, 3, 224, 224, device=dev, generator=g0).to(memory_format=MF)
y = torch.randint(0, 1000, (32,), device=dev, generator=g0)
cur = torch.cuda.current_stream()
side = torch.cuda.Stream()


def fb():
    opt.zero_grad(set_to_none=False)
    with torch.autocast(device_type='cuda', dtype=torch.bfloat16):
        loss = F.cross_entropy(model(x), y, label_smoothing=0.1)
    loss.backward()
    return loss


def update():
    if pre is not None:
        pre.step()
    opt.step()


def on_side(fn):
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        out = fn()
    cur.wait_stream(side)
    return out


if os.environ.get('GTS'):
    from distributed_kfac_pytorch_amd.graphs import GraphedTrainStep

    def step_fn():
        loss = fb()
        update()
        return loss
    fac = int(os.environ.get('FAC', '1000'))
    inv = int(os.environ.get('INV', '1000'))
    if pre is not None:
        pre.param_groups[0]['factor_update_freq'] = fac
        pre.param_groups[0]['inv_update_freq'] = inv
    gts = GraphedTrainStep(step_fn, preconditioner=pre, optimizers=[opt], warmup=int(os.environ.get('WARM', '2')))
    def snap(tag):
        if not os.environ.get('DIAG'):
            return
        torch.cuda.synchronize()

        def mx(ts):
            return max(float(t.float().abs().max()) for t in ts)
        f = pre.fused
        print(tag, 'A %.3g' % mx([l.state['A'] for l in pre.layers]),
              'G %.3g' % mx([l.state['G'] for l in pre.layers]),
              'eig %.3g' % mx([pre.plan.eig_arena]),
              'QG %.3g' % mx([b.QG.t for b in f.bufs]), 'QA %.3g' % mx([b.QA.t for b in f.bufs]),
              'Dt %.3g' % mx([b.Dt for b in f.bufs if b.Dt is not None]),
              'Gct %.3g' % mx([b.Gct.t for b in f.bufs]),
              'grad %.3g' % mx([p.grad for p in model.parameters()]),
              'kl %.4g' % float(f.kl), 'step', pre.param_groups[0]['step'], flush=True)

    def gmax():
        torch.cuda.synchronize()
        worst = sorted(((float(p.grad.float().abs().max()), n) for n, p in model.named_parameters()
                        if p.grad is not None), reverse=True)
        return worst[:3]

    def poke(kind, fillv):
        """Hand freed blocks of many sizes a recognisable value (1e30-ish)."""
        if kind in ('alloc', 'allocside'):
            st = torch.cuda.current_stream() if kind == 'alloc' else gts.side
            with torch.cuda.stream(st):
                ts = [torch.full((n,), fillv, device=dev) for n in
                      (128, 1024, 16384, 262144, 1 << 20, 4 << 20, 16 << 20, 64 << 20)]
                del ts
        torch.cuda.synchronize()

    for _ in range(int(os.environ.get('PRESTEPS', '0'))):
        gts()
    if os.environ.get('POKE'):
        print('before poke', gmax(), flush=True)
        poke(os.environ['POKE'], 1.2345e30)
        for k in range(3):
            gts()
            print('after poke replay', k, gmax(), flush=True)
        sys.exit(0)
    snap('presteps')
    if os.environ.get('PREPARE') == 'manual':
        # gts.prepare() unrolled: plain probe at step 1, factor probe at step 10
        p = pre.param_groups[0]
        saved = p['step']
        for kind, s in (('plain', 1), ('factor', 10)):
            for k in range(gts.warmup + 1):
                p['step'] = s
                gts()
                snap('prep %s %d (graphs %d)' % (kind, k, len(gts.graphs)))
        p['step'] = saved
    elif os.environ.get('PREPARE'):
        gts.prepare()
    snap('prepared')
    if os.environ.get('START'):
        pre.param_groups[0]['step'] = int(os.environ['START'])
    for i in range(int(os.environ.get('NSTEPS', '12'))):
        loss = gts()
        if i < int(os.environ.get('DIAG_STEPS', '0')):
            snap('window %d' % i)
        if os.environ.get('SYNC'):
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    kl = float(pre.fused.kl) if pre is not None else 0.0
    pmax = max(float(p.abs().max()) for p in model.parameters())
    print('final gts prepare=%s' % os.environ.get('PREPARE', ''), 'loss %.4f' % float(loss),
          'kl %.4g' % kl, 'param max %.3g' % pmax, 'replays', gts.replays, 'eager', gts.eager_steps,
          flush=True)
    sys.exit(0)
for _ in range(3):
    on_side(fb)
    update()
torch.cuda.synchronize()
WHOLE = bool(os.environ.get('WHOLE'))
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph, stream=side):
    loss = fb()
    if WHOLE:
        update()
SYNC = os.environ.get('SYNC', '')   # '', 'all', 'after_replay', 'after_kfac', 'after_opt'
EAGER_AT = int(os.environ.get('EAGER_AT', '-1'))   # eager work between replays
EAGER_MODE = os.environ.get('EAGER_MODE', 'full')  # full | fb | inv | sgd


def eager_inverse():
    p = pre.param_groups[0]
    pre.compute_inverses(damping=p['damping'])
    pre._eigendata_updated()


for i in range(int(os.environ.get('NSTEPS', '6'))):
    if i == EAGER_AT and pre is not None:
        saved = pre.param_groups[0]['step']
        if EAGER_MODE == 'full':
            pre.param_groups[0]['step'] = 0
            on_side(fb)
            on_side(update)
        elif EAGER_MODE == 'fb':
            on_side(fb)
        elif EAGER_MODE == 'inv':
            on_side(eager_inverse)
        elif EAGER_MODE == 'sgd':
            on_side(fb)
            on_side(opt.step)
        torch.cuda.synchronize()
        pre.param_groups[0]['step'] = saved + 1
        print('eager', EAGER_MODE, 'at', i, 'kl', float(pre.fused.kl), flush=True)
        continue
    on_side(graph.replay)
    if SYNC in ('all', 'after_replay'):
        torch.cuda.synchronize()
    if WHOLE:
        if pre is not None:
            pre.param_groups[0]['step'] += 1
    else:
        if pre is not None:
            pre.step()
        if SYNC in ('all', 'after_kfac'):
            torch.cuda.synchronize()
        opt.step()
    if SYNC in ('all', 'after_opt'):
        torch.cuda.synchronize()
torch.cuda.synchronize()
kl = float(pre.fused.kl) if pre is not None else 0.0
pmax = max(float(p.abs().max()) for p in model.parameters())
print('final sync=%s' % SYNC, 'loss %.4f' % float(loss), 'kl %.4g' % kl, 'param max %.3g' % pmax,
      flush=True)
