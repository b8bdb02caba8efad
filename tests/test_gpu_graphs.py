"""Whole-step hipGraph capture (graphs.GraphedTrainStep) vs eager execution."""
import pytest
import torch
import torch.nn.functional as F

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd import graphs
from distributed_kfac_pytorch_amd.models import resnet_cifar

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def deterministic_convs():
    # MIOpen's benchmark mode may pick different convolution algorithms in the
    # eager and graphed runs (different rounding, amplified by the K-FAC
    # inverse steps); compare runs on the same deterministic algorithms
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    yield
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev


def _train(use_graphs, steps=25, precision='fp32', segmented=False, set_to_none=False, lag=0,
           amp=True, hybrid=False, early=False):
    torch.manual_seed(0)
    m = resnet_cifar.resnet20().cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    pre = kfac.KFAC(m, factor_update_freq=2, inv_update_freq=10, lr=0.05,
                    precond_precision=precision, compute_factor_in_hook=segmented,
                    inverse_lag=lag)
    pre.early_inverse = early
    g = torch.Generator(device='cuda').manual_seed(3)
    xs = [torch.randn(16, 3, 32, 32, device='cuda', generator=g) for _ in range(steps)]
    ys = [torch.randint(0, 10, (16,), device='cuda', generator=g) for _ in range(steps)]
    x = torch.empty_like(xs[0]).contiguous(memory_format=torch.channels_last)
    y = torch.empty_like(ys[0])

    def step_fn():
        opt.zero_grad(set_to_none=set_to_none)
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        pre.step()
        opt.step()
        return loss

    def fb():
        opt.zero_grad(set_to_none=set_to_none if hybrid else False)
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        return loss

    def update():
        pre.step()
        opt.step()

    if segmented:
        step = graphs.GraphedTrainStep(None, pre, [opt], warmup=1, enabled=use_graphs,
                                       forward_backward=fb, communicate=lambda: None,
                                       update=update)
    elif hybrid:
        step = graphs.GraphedTrainStep(step_fn, pre, [opt], warmup=1, enabled=use_graphs,
                                       forward_backward=fb, update=update)
    else:
        step = graphs.GraphedTrainStep(step_fn, pre, [opt], warmup=1, enabled=use_graphs)
    losses = []
    for i in range(steps):
        x.copy_(xs[i])
        y.copy_(ys[i])
        losses.append(step().item())
    return losses, [p.detach().clone() for p in m.parameters()], step


def _pdiff(pa, pb):
    num = sum((a - b).norm() ** 2 for a, b in zip(pa, pb)) ** 0.5
    den = sum(a.norm() ** 2 for a in pa) ** 0.5
    return (num / den).item()


def test_graphed_matches_eager():
    # 14 steps (bf16 autocast): eager inverse steps 0 and 10, factor steps,
    # plain steps.  With MIOpen's deterministic algorithms every K-FAC kernel
    # is now bitwise reproducible -- the eigensolver's back-transformation
    # sums its split-K slabs in a fixed order (round 3 used f32 atomics and
    # needed a 0.5 % / 20x-noise budget here) -- so eager runs are bitwise
    # equal and the graphed run matches them to 1e-5.
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        le, pe, se = _train(False, steps=14)
        le2, pe2, _ = _train(False, steps=14)
        lg, pg, sg = _train(True, steps=14)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert sg.replays > 0 and len(sg.graphs) == 2      # 'plain' and 'factor' graphs
    assert se.replays == 0
    assert le == le2 and _pdiff(pe, pe2) == 0.0, (le, le2)
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (le, lg)
    assert _pdiff(pe, pg) <= 1e-5, _pdiff(pe, pg)


def test_hybrid_inverse_steps_replay_their_forward_backward():
    """Single-segment trainer that also names forward_backward / update (the
    one-GPU bench): inverse steps 10 and 20 run their forward/backward with the
    factors inside the hooks (KFAC.hook_factors) -- eagerly at step 10 (warm-up),
    as a captured 'invfb' graph at step 20 -- and only the update eagerly.
    Matches the all-eager run, whose factors are computed in step()."""
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        le, pe, _ = _train(False, steps=25, amp=False)
        lh, ph, sh = _train(True, steps=25, amp=False, hybrid=True)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert sh.hybrid and sh.replays > 0
    assert any(k[0] == 'invfb' for k in sh.graphs), list(sh.graphs)
    assert sh.pre.early_inverse_launches == 0
    assert not sh.pre.compute_factor_in_hook        # restored after each inverse step
    for a, b in zip(le, lh):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(a)), (le, lh)
    assert _pdiff(pe, ph) <= 1e-6, _pdiff(pe, ph)


def test_early_inverse_update_matches_one_batch_solve():
    """Hybrid trainer with the opt-in early inverse update (resnet20's five
    576^2 A factors -- layer3 -- are the solve's leading group: updated
    at the first gradient hook of the inverse step's eager
    forward/backward and solved from there on the eigensolver's worker
    stream, joined in step()) against the same trainer replaying an 'invfb'
    graph and solving every factor in step(): same factors, the eigendata of
    the same kernels."""
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        lo, po, so = _train(True, steps=25, amp=False, hybrid=True, early=False)
        le, pe, se = _train(True, steps=25, amp=False, hybrid=True, early=True)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert so.pre.early_inverse_launches == 0 and se.pre.early_inverse_launches == 2
    assert any(k[0] == 'invfb' for k in so.graphs)
    assert not any(k[0] == 'invfb' for k in se.graphs)
    for a, b in zip(lo, le):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(a)), (lo, le)
    assert _pdiff(po, pe) <= 1e-6, _pdiff(po, pe)
    # eigenvalues (eigenvectors of clustered eigenvalues may rotate within the
    # cluster between batch compositions; the preconditioned steps above agree)
    for lo_, le_ in zip(so.pre.layers, se.pre.layers):
        for key in ('dA', 'dG'):
            a, b = lo_.state[key].float(), le_.state[key].float()
            assert (a - b).abs().max().item() <= 1e-4 * max(1.0, a.abs().max().item()), key


def _check_losses(le, le2, lg, rel):
    for a, a2, b in zip(le, le2, lg):
        assert abs(a - b) <= max(rel * max(1.0, abs(a)), 4 * abs(a - a2)), (le, le2, lg)


def test_graphed_equals_eager_deterministic():
    """With the deterministic SYRK (partial tiles, fixed-order reduction) and
    MIOpen's deterministic algorithms in fp32, eager runs are bitwise
    reproducible and the graphed run matches them to 1e-6 (no noise budget)."""
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        le, pe, _ = _train(False, steps=14, amp=False)
        le2, pe2, _ = _train(False, steps=14, amp=False)
        lg, pg, sg = _train(True, steps=14, amp=False)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert sg.replays > 0
    assert le == le2 and _pdiff(pe, pe2) == 0.0, (le, le2)
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(a)), (le, lg)
    assert _pdiff(pe, pg) <= 1e-6, _pdiff(pe, pg)


def test_segmented_graphs_match_eager():
    """forward/backward graph + eager communicate + update graph (the
    multi-rank bench layout), factors computed inside the captured hooks."""
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        le, pe, _ = _train(False, steps=14, segmented=True)
        le2, pe2, _ = _train(False, steps=14, segmented=True)
        ls, ps, ss = _train(True, steps=14, segmented=True)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert ss.replays > 0 and len(ss.graphs) == 4      # fb/update x plain/factor
    assert le == le2 and _pdiff(pe, pe2) == 0.0, (le, le2)
    for a, b in zip(le, ls):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (le, ls)
    assert _pdiff(pe, ps) <= 1e-5, _pdiff(pe, ps)


def test_graphed_set_to_none_matches_eager():
    """zero_grad(set_to_none=True): the graph owns its gradients; eager
    inverse steps allocate their own; K-FAC gathers by value from either."""
    le, pe, _ = _train(False, steps=14, set_to_none=True)
    le2, pe2, _ = _train(False, steps=14, set_to_none=True)
    lg, pg, sg = _train(True, steps=14, set_to_none=True)
    assert sg.replays > 0
    _check_losses(le, le2, lg, 5e-3)
    noise, diff = _pdiff(pe, pe2), _pdiff(pe, pg)
    assert diff < max(5e-3, 20 * noise), (diff, noise)


@pytest.mark.parametrize('segmented', [False, True])
def test_graphed_lagged_inverses_match_eager(segmented):
    """KFAC(inverse_lag=4): the solves of steps 10 and 20 run on a side stream
    from a host thread while graphs replay; they are stored at steps 14 and 24
    (eager steps).  Graphed and eager runs agree."""
    le, pe, _ = _train(False, steps=25, lag=4, segmented=segmented)
    le2, pe2, _ = _train(False, steps=25, lag=4, segmented=segmented)
    lg, pg, sg = _train(True, steps=25, lag=4, segmented=segmented)
    assert sg.replays > 0 and sg.eager_steps == 5     # 0, 10, 14, 20, 24
    # 25 bf16-autocast steps with three inverse updates amplify the run-to-run
    # noise (see test_graphed_matches_eager): 1 % or 4x the eager spread
    _check_losses(le, le2, lg, 1e-2)
    noise, diff = _pdiff(pe, pe2), _pdiff(pe, pg)
    assert diff < max(1e-2, 20 * noise), (diff, noise)


def _train_split(use_graphs, steps=12, phased=False):
    """resnet_tiny, fp32, deterministic: backward in two graph segments
    (parallel/overlap.SplitBackward) and optionally the phased K-FAC update."""
    from distributed_kfac_pytorch_amd.models import resnet
    from distributed_kfac_pytorch_amd.parallel.overlap import SplitBackward
    torch.manual_seed(0)
    m = resnet.resnet_tiny(num_classes=10).cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    pre = kfac.KFAC(m, factor_update_freq=2, inv_update_freq=10, lr=0.05,
                    compute_factor_in_hook=True)
    g = torch.Generator(device='cuda').manual_seed(3)
    xs = [torch.randn(8, 3, 32, 32, device='cuda', generator=g) for _ in range(steps)]
    ys = [torch.randint(0, 10, (8,), device='cuda', generator=g) for _ in range(steps)]
    x = torch.empty_like(xs[0]).contiguous(memory_format=torch.channels_last)
    y = torch.empty_like(ys[0])
    sb = SplitBackward(m, lambda out: F.cross_entropy(out, y), lambda: x)

    def update():
        pre.step()
        opt.step()
    step = graphs.GraphedTrainStep(None, pre, [opt], warmup=1, enabled=use_graphs,
                                   forward_backward=sb.segments, communicate=sb.communicate,
                                   update=update, phased_update='force' if phased else False)
    losses = []
    for i in range(steps):
        x.copy_(xs[i])
        y.copy_(ys[i])
        losses.append(step().item())
    return losses, [p.detach().clone() for p in m.parameters()], step


@pytest.mark.parametrize('phased', [False, True])
def test_split_backward_segments_graphed(phased):
    """Two backward graph segments (the overlapped all-reduce layout) and the
    phased K-FAC update (the MEM/HYBRID layout) replay exactly like eager."""
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        le, pe, _ = _train_split(False, phased=phased)
        lg, pg, sg = _train_split(True, phased=phased)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert sg.replays > 0
    keys = {k[0] for k in sg.graphs}
    assert {'fb', 'fb1'} <= keys, keys
    if phased:
        assert {'upd_pre', 'upd_post'} <= keys, keys
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(a)), (le, lg)
    assert _pdiff(pe, pg) <= 1e-6, _pdiff(pe, pg)


def _train_fp16(use_graphs, steps=14, overflow_at=None):
    """fp16 autocast + GradScaler + fused SGD (found_inf consumed on the
    device): K-FAC's G unscale / non-finite filter is device-side, so the
    whole step -- scaler.unscale_, KFAC.step, scaler.step, scaler.update --
    is capturable."""
    torch.manual_seed(0)
    m = resnet_cifar.resnet20().cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9, fused=True)
    scaler = torch.amp.GradScaler('cuda', init_scale=2.0 ** 12)
    pre = kfac.KFAC(m, factor_update_freq=2, inv_update_freq=10, lr=0.05, grad_scaler=scaler)
    g = torch.Generator(device='cuda').manual_seed(3)
    xs = [torch.randn(16, 3, 32, 32, device='cuda', generator=g) for _ in range(steps)]
    ys = [torch.randint(0, 10, (16,), device='cuda', generator=g) for _ in range(steps)]
    x = torch.empty_like(xs[0]).contiguous(memory_format=torch.channels_last)
    y = torch.empty_like(ys[0])
    mult = torch.ones((), device='cuda')     # 1e30 at overflow_at: inf gradients in fp16

    def step_fn():
        opt.zero_grad(set_to_none=False)
        with torch.autocast('cuda', dtype=torch.float16):
            loss = F.cross_entropy(m(x), y)
        scaler.scale(loss * mult).backward()
        scaler.unscale_(opt)
        pre.step()
        scaler.step(opt)
        scaler.update()
        return loss

    step = graphs.GraphedTrainStep(step_fn, pre, [opt], warmup=1, enabled=use_graphs)
    losses = []
    for i in range(steps):
        x.copy_(xs[i])
        y.copy_(ys[i])
        mult.fill_(1e30 if i == overflow_at else 1.0)
        losses.append(step().item())
    return losses, [p.detach().clone() for p in m.parameters()], step, pre


def test_fp16_gradscaler_step_captures():
    le, pe, _, _ = _train_fp16(False)
    lg, pg, sg, pre = _train_fp16(True)
    assert sg.replays > 0 and {'plain', 'factor'} <= {k[1] for k in sg.graphs}, sg.graphs.keys()
    assert all(torch.isfinite(p).all() for p in pg)
    for a, b in zip(le, lg):
        assert abs(a - b) < 3e-2 * max(1.0, abs(a)), (le, lg)
    assert _pdiff(pe, pg) < 2e-2


def test_fp16_overflow_step_filtered_on_device():
    """An overflowing step (inf gradients, replayed from a graph) leaves the
    parameters and the G factors finite: the scaler skips the update and
    K-FAC's device-side filter drops the non-finite G contribution."""
    _, pg, sg, pre = _train_fp16(True, steps=14, overflow_at=12)   # step 12: a factor step
    assert sg.replays > 0
    assert all(torch.isfinite(p).all() for p in pg)
    for l in pre.layers:
        assert torch.isfinite(l.state['G']).all() and torch.isfinite(l.state['A']).all()
