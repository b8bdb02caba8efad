"""Debug: which state turns non-finite in the first graph replay after the
eager inverse step (bench.py flow, single GPU)."""
import os
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, os.getcwd())
import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.models import resnet  # noqa: E402
from distributed_kfac_pytorch_amd import graphs  # noqa: E402

dev = torch.device('cuda')
torch.manual_seed(1234)
torch.backends.cudnn.benchmark = True
model = resnet.get_model('resnet50').to(dev).to(memory_format=torch.channels_last)
opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9, weight_decay=5e-5)
pre = kfac.KFAC(model, damping=1e-3, factor_decay=0.95, factor_update_freq=int(os.environ.get('FAC', '10')), inv_update_freq=int(os.environ.get('INV', '100')),
                kl_clip=None if os.environ.get('NOKL') else 1e-3, lr=0.0125,
                distribute_layer_factors=False,
                precond_precision=os.environ.get('PREC', 'bf16x3'),
                fused_precondition=not os.environ.get('NOFUSED'),
                compute_factor_in_hook=bool(os.environ.get('SEG')))
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(32, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev, generator=g)


def train_step():
    opt.zero_grad(set_to_none=False)
    with torch.autocast(device_type='cuda', dtype=torch.bfloat16):
        loss = F.cross_entropy(model(x), y, label_smoothing=0.1)
    loss.backward()
    pre.step()
    opt.step()
    return loss


def report(tag):
    torch.cuda.synchronize()
    bad = []
    for name, p in model.named_parameters():
        if not torch.isfinite(p).all():
            bad.append('param ' + name)
        if p.grad is not None and not torch.isfinite(p.grad).all():
            bad.append('grad ' + name)
    for i, l in enumerate(pre.layers):
        for k, v in l.state.items():
            if torch.is_tensor(v) and not torch.isfinite(v).all():
                bad.append('state %d %s' % (i, k))
        if l.pgrad_buffer is not None and not torch.isfinite(l.pgrad_buffer).all():
            bad.append('pgrad %d' % i)
    f = pre.fused
    if f is None:
        gmax = max(float(p.grad.abs().max()) for p in model.parameters() if p.grad is not None)
        print(tag, '|grad|', gmax, 'bad', len(bad), bad[:6], flush=True)
        return
    for i, b in enumerate(f.bufs):
        for nm in ('QG', 'QGt', 'QA', 'QAt', 'Gct', 'T1', 'T2t', 'T3'):
            t = getattr(b, nm).t
            if not torch.isfinite(t.float()).all():
                bad.append('fused %d %s' % (i, nm))
        if b.Dt is not None and not torch.isfinite(b.Dt).all():
            bad.append('fused %d Dt' % i)
    gmax = max(float(p.grad.abs().max()) for p in model.parameters() if p.grad is not None)
    pmax = max(float(l.pgrad_buffer.abs().max()) for l in pre.layers)
    cmax = max(float(b.Gct.t.float().abs().max()) for b in f.bufs)
    print(tag, 'kl', float(f.kl), '|grad|', gmax, '|pgrad|', pmax, '|Gct|', cmax, 'bad', len(bad),
          bad[:6], flush=True)


if os.environ.get('SEG'):
    def fb():
        opt.zero_grad(set_to_none=False)
        with torch.autocast(device_type='cuda', dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y, label_smoothing=0.1)
        loss.backward()
        return loss

    def upd():
        pre.step()
        opt.step()
    comm = (lambda: torch.cuda.synchronize()) if os.environ.get('SEG_SYNC') else None
    step = graphs.GraphedTrainStep(None, pre, [opt], forward_backward=fb, update=upd,
                                   communicate=comm)
    step._update_capturable = lambda kind: bool(os.environ.get('SEG_CAPTURE_UPDATE'))
else:
    step = graphs.GraphedTrainStep(train_step, pre, [opt], enabled=not os.environ.get('NOGRAPH'))
def gptrs():
    return tuple(p.grad.data_ptr() if p.grad is not None else 0 for p in model.parameters())


hist = []
for i in range(10):
    step()
    hist.append((i, step.replays, hash(gptrs())))
    if not os.environ.get('NOSYNC') or os.environ.get('WARMUP_REPORT'):
        report('warmup %d replays %d' % (i, step.replays))
step.prepare()
torch.cuda.synchronize()
hist.append(('prepare', step.replays, hash(gptrs())))
print('grad ptr history', hist, flush=True)


def rng(t, name):
    st = t.untyped_storage()
    return (st.data_ptr(), st.data_ptr() + st.nbytes(), name)


ranges = []
for n_, p_ in model.named_parameters():
    ranges.append(rng(p_, 'param ' + n_))
    if p_.grad is not None:
        ranges.append(rng(p_.grad, 'grad ' + n_))
    st_ = opt.state.get(p_, {})
    if 'momentum_buffer' in st_ and st_['momentum_buffer'] is not None:
        ranges.append(rng(st_['momentum_buffer'], 'mom ' + n_))
for n_, b_ in model.named_buffers():
    ranges.append(rng(b_, 'buf ' + n_))
if pre.fused is not None:
    ranges.append(rng(pre.fused.kl, 'kfac kl'))
    for i_, b_ in enumerate(pre.fused.bufs):
        for nm in ('QG', 'QGt', 'QA', 'QAt', 'Gct', 'T1', 'T2t', 'T3'):
            ranges.append(rng(getattr(b_, nm).t, 'kfac %d %s' % (i_, nm)))
ranges.append(rng(pre.plan.grad_arena, 'kfac pgrad arena'))
ranges.append(rng(pre.plan.eig_arena, 'kfac eig arena'))
for i_, l_ in enumerate(pre.layers):
    for k_, v_ in l_.state.items():
        if torch.is_tensor(v_):
            ranges.append(rng(v_, 'kfac state %d %s' % (i_, k_)))
uniq = {}
for a_, b_, n_ in ranges:
    uniq.setdefault((a_, b_), n_)
rs = sorted((a_, b_, n_) for (a_, b_), n_ in uniq.items())
over = []
for (a1, b1, n1), (a2, b2, n2) in zip(rs, rs[1:]):
    if a2 < b1:
        over.append((n1, n2))
print('overlapping storages:', len(over), over[:10], flush=True)
ptrs = {n: (p.grad.data_ptr() if p.grad is not None else None) for n, p in model.named_parameters()}
print('after prepare kl', float(pre.fused.kl) if pre.fused is not None else None, 'replays', step.replays, flush=True)
pre.param_groups[0]['step'] = int(os.environ.get('START', '0'))
import gc, time  # noqa: E401,E402
BETWEEN = os.environ.get('BETWEEN', '')
for i in range(int(os.environ.get('NSTEPS', '4'))):
    loss = step()
    if BETWEEN == 'sleep':
        time.sleep(0.05)
    elif BETWEEN == 'gc':
        torch.cuda.synchronize()
        gc.collect()
    elif BETWEEN == 'read':
        torch.cuda.synchronize()
        _ = [float(p.grad.abs().max()) for p in model.parameters()]
    if not os.environ.get('NOSYNC'):
        report('after step %d (loss %.4f)' % (i, float(loss)))
report('final (loss %.4f)' % float(loss))
moved = [n for n, p in model.named_parameters() if (p.grad.data_ptr() if p.grad is not None else None) != ptrs[n]]
print('grads moved since prepare:', len(moved), moved[:5], flush=True)
