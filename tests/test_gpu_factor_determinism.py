"""Deterministic factor covariances (csrc/factors.hip: per-split partial
tiles reduced in a fixed order, no f32 atomics): the same activations give
bitwise-equal factors, on the grouped (bf16 channels_last) and per-factor
(fp32 NCHW) paths, and both match an fp64 reference."""
import pytest
import torch
import torch.nn.functional as F

from distributed_kfac_pytorch_amd.ops import factors

pytestmark = pytest.mark.gpu


class _Geom(object):
    def __init__(self, k, s, p):
        self.kh = self.kw = k
        self.sh = self.sw = s
        self.ph = self.pw = p
        self.dh = self.dw = 1


def _ref_cov(x, k, s, p, has_bias):
    cols = F.unfold(x.double(), k, padding=p, stride=s)          # (B, C*k*k, L)
    P = cols.transpose(1, 2).reshape(-1, cols.shape[1])
    if has_bias:
        P = torch.cat([P, torch.ones(P.shape[0], 1, dtype=P.dtype, device=P.device)], 1)
    return P.t() @ P / P.shape[0]


@pytest.mark.parametrize('dtype,cl', [(torch.bfloat16, True), (torch.float32, False)])
def test_factor_update_bitwise_reproducible(dtype, cl):
    g = torch.Generator(device='cuda').manual_seed(5)
    x = torch.randn(16, 64, 28, 28, device='cuda', generator=g).to(dtype)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    geom = _Geom(3, 1, 1)
    n = 64 * 9 + 1
    src = factors.FactorSource(x, geom, True, 1.0)
    rows = src.rows[0]
    src.scale = 1.0 / rows
    outs = []
    for _ in range(3):
        st = torch.zeros(n, n, device='cuda')
        if cl:
            st = factors.update_factors_grouped([(st, [src], torch.float32)], 0.0)[0]
        else:
            st = factors.update_factor(st, [src], 0.0, torch.float32)
        outs.append(st.clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    ref = _ref_cov(x, 3, 1, 1, True)
    err = ((outs[0].double() - ref).norm() / ref.norm()).item()
    assert err < (2e-3 if dtype == torch.bfloat16 else 1e-5), err


@pytest.mark.parametrize('cl', [True, False])
def test_fp32_few_channel_split_factor(cl):
    """ResNet's conv1 input (fp32, C = 3, 7x7 / 2): the grouped path takes it
    as fp16 hi / lo planes (kfac_split_f16) -- bitwise reproducible, within
    fp32-level error of the fp64 covariance and of the generic fp32 SYRK."""
    g = torch.Generator(device='cuda').manual_seed(7)
    x = torch.randn(8, 3, 64, 64, device='cuda', generator=g) * 2.5 + 0.3
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    geom = _Geom(7, 2, 3)
    n = 3 * 49
    src = factors.FactorSource(x, geom, False, 1.0)
    src.scale = 1.0 / src.rows[0]
    before = factors.split_launches
    outs = []
    for _ in range(3):
        st = torch.zeros(n, n, device='cuda')
        outs.append(factors.update_factors_grouped([(st, [src], torch.float32)], 0.0)[0].clone())
    assert factors.split_launches == before + 3
    generic = factors.update_factor(torch.zeros(n, n, device='cuda'), [src], 0.0, torch.float32)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert torch.equal(outs[0], outs[0].t())
    ref = _ref_cov(x, 7, 2, 3, False)
    err = ((outs[0].double() - ref).norm() / ref.norm()).item()
    gerr = ((generic.double() - ref).norm() / ref.norm()).item()
    assert err < 2e-6 and err < 20 * max(gerr, 1e-8), (err, gerr)


def test_multi_source_factor_reproducible():
    """Several sources of one factor (gradient accumulation): the partials of
    every (source, split) are summed in a fixed order."""
    g = torch.Generator(device='cuda').manual_seed(6)
    xs = [torch.randn(8, 32, 14, 14, device='cuda', generator=g).to(torch.bfloat16)
          .contiguous(memory_format=torch.channels_last) for _ in range(3)]
    geom = _Geom(3, 1, 1)
    srcs = [factors.FactorSource(x, geom, False, 1.0 / (8 * 14 * 14 * 3)) for x in xs]
    n = 32 * 9
    a = factors.update_factors_grouped([(torch.zeros(n, n, device='cuda'), srcs,
                                         torch.float32)], 0.0)[0].clone()
    b = factors.update_factors_grouped([(torch.zeros(n, n, device='cuda'), srcs,
                                         torch.float32)], 0.0)[0].clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    ref = sum(_ref_cov(x, 3, 1, 1, False) for x in xs) / 3
    assert ((a.double() - ref).norm() / ref.norm()).item() < 2e-3


def test_many_sources_grouped_bitwise():
    """More sources than one tile-reduction job holds (an LSTM at bptt 35
    with accumulate_data: one Linear source per time step): the grouped path
    chains fixed-order reductions, so the factor is bitwise reproducible and
    equals the fp64 sum."""
    g = torch.Generator(device='cuda').manual_seed(8)
    T, B, D = 35, 20, 256
    xs = [torch.randn(B, D, device='cuda', generator=g).to(torch.bfloat16) for _ in range(T)]
    srcs = [factors.linear_source(x, True) for x in xs]
    for s in srcs:
        s.scale = 1.0 / (B * T)
    n = D + 1
    outs = []
    for _ in range(3):
        st = torch.zeros(n, n, device='cuda')
        st = factors.update_factors_grouped([(st, srcs, torch.float32)], 0.0)[0]
        outs.append(st.clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    P = torch.cat([torch.cat([x.double(), torch.ones(B, 1, dtype=torch.float64, device='cuda')], 1)
                   for x in xs], 0)
    ref = P.t() @ P / (B * T)
    err = ((outs[0].double() - ref).norm() / ref.norm()).item()
    assert err < 1e-5, err


def test_lstm_lm_factors_bitwise():
    """The LSTM LM (bptt 35, accumulate_data=True, bf16 autocast): two
    identical K-FAC factor steps give bitwise-equal factors for every layer
    (round 2 fell back to f32-atomic SYRKs past 8 sources).  The 16-bit
    sources (the gate Linears' inputs x_t and every grad output) go through
    the grouped path; the hidden-state inputs h_t stay fp32 under autocast
    (c_t is fp32, h_t = o_t tanh(c_t)), so the hh Linears' A factors take the
    per-factor fp32 path -- chained, deterministic too."""
    import distributed_kfac_pytorch_amd as kfac
    from distributed_kfac_pytorch_amd.models import lstm_lm

    def run():
        torch.manual_seed(0)
        model = lstm_lm.LSTMModel(1000, 128, 128, 2, dropout=0.0).cuda()
        pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=1000, accumulate_data=True,
                        skip_layers=['embedding', 'linear'])
        x = torch.randint(0, 1000, (35, 20), device='cuda',
                          generator=torch.Generator(device='cuda').manual_seed(1))
        h = model.init_hidden(20)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out, _ = model(x, h)
        out.float().sum().backward()
        calls = []
        orig = factors.update_factor
        factors.update_factor = lambda *a, **k: calls.append(1) or orig(*a, **k)
        try:
            pre.compute_factors(alpha=0.95)
        finally:
            factors.update_factor = orig
        # 2 layers x hh Linear: the A factors over the fp32 hidden states
        assert len(calls) <= 4, 'more LSTM factors than the fp32 ones left the grouped path'
        torch.cuda.synchronize()
        return [(l.state['A'].clone(), l.state['G'].clone()) for l in pre.layers]

    a, b = run(), run()
    assert len(a) > 0
    for (A1, G1), (A2, G2) in zip(a, b):
        assert torch.equal(A1, A2) and torch.equal(G1, G2)


def _train_factors(early, graphed, steps=7, hook=False):
    import distributed_kfac_pytorch_amd as kfac
    from distributed_kfac_pytorch_amd import graphs
    from distributed_kfac_pytorch_amd.models import resnet
    torch.manual_seed(0)
    m = resnet.resnet_tiny(num_classes=10).cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    # damped-inverse path: bitwise reproducible inputs to every later step
    pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=4, lr=0.05, damping=0.003,
                    use_eigen_decomp=False, early_factors=early, compute_factor_in_hook=hook)
    g = torch.Generator(device='cuda').manual_seed(3)
    xs = [torch.randn(8, 3, 32, 32, device='cuda', generator=g) for _ in range(steps)]
    ys = [torch.randint(0, 10, (8,), device='cuda', generator=g) for _ in range(steps)]
    x = torch.empty_like(xs[0]).contiguous(memory_format=torch.channels_last)
    y = torch.empty_like(ys[0])

    def step_fn():
        opt.zero_grad(set_to_none=False)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        pre.step()
        opt.step()
        return loss

    step = graphs.GraphedTrainStep(step_fn, pre, [opt], warmup=1, enabled=graphed)
    for i in range(steps):
        x.copy_(xs[i])
        y.copy_(ys[i])
        step()
    torch.cuda.synchronize()
    return ([l.state[w].clone() for l in pre.layers for w in ('A', 'G')],
            [p.detach().clone() for p in m.parameters()], pre, step)


@pytest.mark.parametrize('graphed', [False, True])
def test_early_factors_bitwise(graphed):
    """KFAC(early_factors=True) computes the A factors on a side stream from
    the first gradient hook, under the backward: the factors and the whole
    trajectory are bitwise those of computing every factor in step()."""
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        f0, p0, _, _ = _train_factors(False, graphed)
        f1, p1, pre, step = _train_factors(True, graphed)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert pre._factor_stream is not None and pre._early_a is None
    if graphed:
        assert step.replays > 0
    for a, b in zip(f0, f1):
        assert torch.equal(a, b), (a - b).abs().max()
    for a, b in zip(p0, p1):
        assert torch.equal(a, b), (a - b).abs().max()


def test_early_factors_survive_counter_rewinds():
    """GraphedTrainStep.prepare() and a bench restarting its window rewind
    the K-FAC step counter: with one forward per step() that is not micro-
    batching, so early_factors stays on (forwards are counted between step()
    calls, not per counter value) and the eager inverse step still launches
    the A factors early."""
    import warnings
    import distributed_kfac_pytorch_amd as kfac
    from distributed_kfac_pytorch_amd import graphs
    from distributed_kfac_pytorch_amd.models import resnet
    torch.manual_seed(0)
    m = resnet.resnet_tiny(num_classes=10).cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    pre = kfac.KFAC(m, factor_update_freq=2, inv_update_freq=4, lr=0.05, damping=0.003,
                    early_factors=True)
    x = torch.randn(8, 3, 32, 32, device='cuda').contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device='cuda')

    def step_fn():
        opt.zero_grad(set_to_none=False)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        pre.step()
        opt.step()
        return loss

    step = graphs.GraphedTrainStep(step_fn, pre, [opt], warmup=1)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        for _ in range(3):
            step()
        step.prepare()
        pre.param_groups[0]['step'] = 0
        launched = pre._early_a_step
        for _ in range(6):
            step()
        torch.cuda.synchronize()
    assert not [x for x in w if 'several forward passes' in str(x.message)]
    assert pre.early_factors
    assert pre._early_a_step is not None and pre._early_a_step != launched


@pytest.mark.parametrize('graphed', [False, True])
def test_hook_factors_grouped_bitwise(graphed):
    """compute_factor_in_hook=True on the GPU (the multi-rank segmented-graph
    mode) saves in the hooks and runs the grouped factor launches from the
    backward's last gradient hook: bitwise the factors and trajectory of
    computing them in step()."""
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        f0, p0, _, _ = _train_factors(False, graphed)
        f1, p1, pre, step = _train_factors(False, graphed, hook=True)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert pre._hook_factors_grouped() and pre._hook_step is not None
    for l in pre.layers:
        assert not l.a_inputs and not l.g_outputs
    for a, b in zip(f0, f1):
        assert torch.equal(a, b), (a - b).abs().max()
    for a, b in zip(p0, p1):
        assert torch.equal(a, b), (a - b).abs().max()


def test_hook_factors_grouped_unused_output():
    """Grouped in-hook factors with a hooked module whose output the loss does
    not use (an aux head in the loss on the first step only): from then on its
    gradient hook never runs, so the backward's 'last hook' never comes;
    step() computes the saved factors instead (with one warning) and the
    factors equal those of computing them in step()."""
    import warnings
    import distributed_kfac_pytorch_amd as kfac

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(32, 64)
            self.b = torch.nn.Linear(64, 10)
            self.aux = torch.nn.Linear(64, 5)

        def forward(self, x):
            h = torch.relu(self.a(x))
            self.aux_out = self.aux(h)        # hooked, never reaches the loss
            return self.b(h)

    def run(hook):
        torch.manual_seed(0)
        m = Net().cuda()
        pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=2, damping=0.003,
                        compute_factor_in_hook=hook)
        g = torch.Generator(device='cuda').manual_seed(4)
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter('always')
            for i in range(4):
                x = torch.randn(16, 32, device='cuda', generator=g)
                loss = F.cross_entropy(m(x), torch.zeros(16, dtype=torch.long, device='cuda'))
                if i == 0:
                    loss = loss + 0.1 * m.aux_out.square().mean()
                loss.backward()
                pre.step()
        torch.cuda.synchronize()
        msgs = [str(x.message) for x in w if 'received no gradient' in str(x.message)]
        return {id(l.module): (l.state['A'], l.state['G']) for l in pre.layers}, pre, m, msgs

    f0, _, m0, _ = run(False)
    f1, pre, m1, msgs = run(True)
    assert pre._hook_factors_grouped() and len(msgs) == 1, msgs
    for l in pre.layers:
        assert not l.a_inputs and not l.g_outputs
    for (mod0, mod1) in zip((m0.a, m0.b, m0.aux), (m1.a, m1.b, m1.aux)):
        A0, G0 = f0[id(mod0)]
        A1, G1 = f1[id(mod1)]
        assert torch.equal(A0, A1)
        assert (G0 is None) == (G1 is None)
        if G0 is not None:
            assert torch.equal(G0, G1)


def test_early_factors_micro_batching_equivalent():
    """early_factors with two forward/backward passes per step (micro-batching,
    accumulate_data=False): no early A launch (it would apply the first
    micro-batch's EMA on top of step()'s), so the factors equal the
    non-early run bitwise."""
    import distributed_kfac_pytorch_amd as kfac
    from distributed_kfac_pytorch_amd.models import resnet

    def run(early):
        torch.manual_seed(0)
        m = resnet.resnet_tiny(num_classes=10).cuda().to(memory_format=torch.channels_last)
        pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=100, damping=0.003,
                        use_eigen_decomp=False, early_factors=early)
        g = torch.Generator(device='cuda').manual_seed(9)
        for _ in range(4):
            for _ in range(2):
                x = torch.randn(8, 3, 32, 32, device='cuda', generator=g).contiguous(
                    memory_format=torch.channels_last)
                y = torch.randint(0, 10, (8,), device='cuda', generator=g)
                with torch.autocast('cuda', dtype=torch.bfloat16):
                    loss = F.cross_entropy(m(x), y) / 2
                loss.backward()
            pre.step()
            m.zero_grad(set_to_none=False)
        torch.cuda.synchronize()
        return [l.state[w].clone() for l in pre.layers for w in ('A', 'G')], pre

    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        f0, _ = run(False)
        f1, pre = run(True)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert pre._early_a_step is None       # never launched early
    for a, b in zip(f0, f1):
        assert torch.equal(a, b), (a - b).abs().max()


@pytest.mark.parametrize('graphed', [False, True])
def test_lstm_lm_hook_factors_grouped_segmented_bitwise(graphed):
    """The LSTM LM (accumulate_data=True, bptt 20) on the multi-rank
    segmented-graph layout (forward/backward graph, eager communicate,
    update graph) with the factors computed in the captured hooks: the
    grouped in-hook path folds every time step's sources into one launch
    sequence at the backward's last gradient hook, and the factors and the
    trajectory are bitwise those of computing the factors in step()."""
    import distributed_kfac_pytorch_amd as kfac
    from distributed_kfac_pytorch_amd import graphs
    from distributed_kfac_pytorch_amd.models import lstm_lm

    def run(hook, use_graphs):
        torch.manual_seed(0)
        m = lstm_lm.LSTMModel(500, 64, 64, 2, dropout=0.0).cuda()
        opt = torch.optim.SGD(m.parameters(), lr=0.5)
        pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=3, damping=0.003,
                        accumulate_data=True, compute_factor_in_hook=hook,
                        skip_layers=['embedding', 'decoder'], use_eigen_decomp=False)
        g = torch.Generator(device='cuda').manual_seed(2)
        xs = [torch.randint(0, 500, (20, 8), device='cuda', generator=g) for _ in range(6)]
        ys = [torch.randint(0, 500, (20, 8), device='cuda', generator=g) for _ in range(6)]
        x, y = torch.empty_like(xs[0]), torch.empty_like(ys[0])

        def fb():
            opt.zero_grad(set_to_none=False)
            with torch.autocast('cuda', dtype=torch.bfloat16):
                out, _ = m(x)
                loss = F.cross_entropy(out.float().view(-1, 500), y.view(-1))
            loss.backward()
            return loss

        def update():
            pre.step()
            opt.step()
        step = None
        if hook:
            step = graphs.GraphedTrainStep(None, pre, [opt], warmup=1, enabled=use_graphs,
                                           forward_backward=fb, communicate=lambda: None,
                                           update=update)
        for i in range(6):
            x.copy_(xs[i])
            y.copy_(ys[i])
            if step is not None:
                step()
            else:            # the plain eager loop, factors in step()
                fb()
                update()
        torch.cuda.synchronize()
        return ([l.state[w].clone() for l in pre.layers for w in ('A', 'G')],
                [p.detach().clone() for p in m.parameters()], pre, step)

    # baseline: eager, factors in step() (a replayed graph runs no Python
    # hook, so the graphed layout needs the in-hook factors)
    f0, p0, _, _ = run(False, False)
    f1, p1, pre, step = run(True, graphed)
    assert pre._hook_factors_grouped() and pre.accumulate_data
    if graphed:
        assert step.replays > 0
    for a, b in zip(f0, f1):
        assert torch.equal(a, b), (a - b).abs().max()
    for a, b in zip(p0, p1):
        assert torch.equal(a, b), (a - b).abs().max()
