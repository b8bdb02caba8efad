"""KFAC public API behaviour on CPU (SURVEY.md Appendix A contract)."""
import copy
import warnings

import pytest
import torch
import torch.nn as nn

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.models import resnet_cifar, resnet, LSTMModel
from tests._oracle_common import SmallNet, build_case, run_steps


def _step(model, pre, x, y):
    model.zero_grad()
    nn.functional.cross_entropy(model(x), y).backward()
    pre.step()


def test_registration_counts():
    assert len(kfac.KFAC(resnet_cifar.resnet20()).layers) == 20
    assert len(kfac.KFAC(resnet_cifar.resnet32()).layers) == 32
    assert len(kfac.KFAC(resnet.resnet50()).layers) == 54


def test_skip_layers_by_module_name():
    from distributed_kfac_pytorch_amd.models import TransformerLM
    lm = TransformerLM(50, d_model=16, n_layers=2, n_heads=2, d_ff=32, max_len=8)
    n_all = len(kfac.KFAC(lm, skip_layers=['embedding']).layers)
    assert n_all == 2 * 4 + 1
    assert len(kfac.KFAC(lm, skip_layers=['embedding', 'head']).layers) == n_all - 1
    assert len(kfac.KFAC(lm, skip_layers=['embedding', 'blocks.0.fc1']).layers) == n_all - 1
    assert len(kfac.KFAC(lm, skip_layers=['embedding', 'blocks.1']).layers) == n_all - 4


def test_skip_layers():
    m = resnet_cifar.resnet20()
    assert len(kfac.KFAC(m, skip_layers='linear').layers) == 19
    assert len(kfac.KFAC(resnet_cifar.resnet20(), skip_layers=['Conv2d']).layers) == 1
    # skipping a container class stops recursion into it
    assert len(kfac.KFAC(resnet_cifar.resnet20(), skip_layers=['sequential']).layers) == 2


def test_embedding_must_be_skipped():
    m = nn.Sequential(nn.Embedding(10, 4), nn.Linear(4, 2))
    with pytest.raises(ValueError):
        kfac.KFAC(m)
    assert len(kfac.KFAC(m, skip_layers=['embedding']).layers) == 1


def test_torch_lstmcell_rejected_and_kfac_lstm_registered():
    with pytest.raises(TypeError):
        kfac.KFAC(nn.Sequential(nn.LSTMCell(4, 4)), skip_layers=[])
    lm = LSTMModel(50, 8, 8, 2, dropout=0.0)
    pre = kfac.KFAC(lm, skip_layers=['embedding'])
    # 2 layers x (ih, hh) LinearMulti + decoder Linear
    assert len(pre.layers) == 5
    names = [type(l).__name__ for l in pre.layers]
    assert names.count('LinearMultiLayer') == 4


def test_frozen_module_not_registered():
    m = SmallNet()
    for p in m.c2.parameters():
        p.requires_grad_(False)
    assert len(kfac.KFAC(m).layers) == 4


def test_invalid_arguments():
    m = SmallNet()
    for kw in [dict(lr=-1), dict(factor_decay=0), dict(factor_decay=1.5), dict(damping=0),
               dict(kl_clip=0), dict(factor_update_freq=0), dict(inv_update_freq=0),
               dict(assignment_strategy='x')]:
        with pytest.raises(ValueError):
            kfac.KFAC(m, **kw)
    with pytest.warns(UserWarning):
        kfac.KFAC(m, factor_update_freq=3, inv_update_freq=10)


def test_compute_factor_in_hook_bit_identical():
    cfg = {'seed': 0, 'batch': 6, 'steps': 3}
    outs = []
    for in_hook in (False, True):
        model, data = build_case(cfg)
        pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=2,
                        compute_factor_in_hook=in_hook)
        outs.append(run_steps(model, pre, data, cfg['steps']))
    for a, b in zip(outs[0][0], outs[1][0]):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


def test_defer_hook_factors_micro_batches():
    """Micro-batched steps with the factors in the hooks (the graphed
    multi-rank examples' mode): deferring all but the last micro-batch gives
    the factors of computing them in step() -- the last micro-batch, one EMA
    update per factor step -- while without deferral every
    micro-batch's pass applies its own EMA update."""
    torch.manual_seed(0)
    base = SmallNet()
    x = torch.randn(8, 3, 8, 8)
    y = torch.randint(0, 10, (8,))
    states = {}
    for mode in ('step', 'deferred', 'every'):
        model = copy.deepcopy(base)
        pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=1,
                        compute_factor_in_hook=(mode != 'step'))
        for _ in range(2):
            model.zero_grad()
            for i in range(2):          # two micro-batches of 4
                ctx = pre.defer_hook_factors() if (mode == 'deferred' and i == 0) else \
                    warnings.catch_warnings()
                with ctx:
                    out = model(x[4 * i:4 * i + 4])
                    (nn.functional.cross_entropy(out, y[4 * i:4 * i + 4]) / 2).backward()
            pre.step()
        states[mode] = [(l.state['A'].clone(), l.state['G'].clone()) for l in pre.layers]
    for (a1, g1), (a2, g2) in zip(states['step'], states['deferred']):
        assert torch.equal(a1, a2) and torch.equal(g1, g2)
    assert any(not torch.equal(a1, a2) for (a1, _), (a2, _) in zip(states['step'],
                                                                    states['every']))


@pytest.mark.parametrize('kw', [dict(precompute_outer_eigen=False), dict(use_eigen_decomp=False),
                                dict(kl_clip=None), dict(factor_dtype=torch.float64),
                                dict(inv_dtype=torch.float64), dict(accumulate_data=True)])
def test_variants_run_and_change_grads(kw):
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': 3})
    ref = copy.deepcopy(model)
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=1, **kw)
    grads, _ = run_steps(model, pre, data, 3)
    model.zero_grad()
    nn.functional.cross_entropy(ref(data[0][0]), data[0][1]).backward()
    plain = [p.grad for p in ref.parameters()]
    assert all(torch.isfinite(g).all() for g in grads[0])
    assert any(not torch.allclose(a, b) for a, b in zip(grads[0], plain))


def test_state_dict_layout_and_roundtrip():
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': 3})
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=2)
    sched = torch.optim.lr_scheduler.LambdaLR(pre, lambda e: 1.0)
    run_steps(model, pre, data, 3)
    sd = pre.state_dict()
    assert set(sd) == {'state', 'param_groups', 'layers'}
    g = sd['param_groups'][0]
    for key in ('damping', 'factor_decay', 'factor_update_freq', 'inv_update_freq', 'kl_clip',
                'lr', 'step', 'initial_lr'):
        assert key in g
    assert g['step'] == 3
    assert all(set(l) == {'A', 'G'} for l in sd['layers'])
    sd_inv = pre.state_dict(include_layer_inverses=True)
    assert {'QA', 'QG', 'dGdA'} <= set(sd_inv['layers'][0])
    model2, _ = build_case({'seed': 1, 'batch': 6, 'steps': 1})
    pre2 = kfac.KFAC(model2, factor_update_freq=1, inv_update_freq=2)
    pre2.load_state_dict(copy.deepcopy(sd))
    assert pre2.param_groups[0]['step'] == 3
    for a, b in zip(pre.layers, pre2.layers):
        assert torch.equal(a.state['A'], b.state['A'])
        assert torch.allclose(a.state['dGdA'], b.state['dGdA'])
    bad = copy.deepcopy(sd)
    bad['layers'] = bad['layers'][:-1]
    with pytest.raises(ValueError):
        pre2.load_state_dict(bad)
    legacy = copy.deepcopy(sd)
    legacy['layers'] = [{'A_factor': l['A'], 'G_factor': l['G']} for l in legacy['layers']]
    pre2.load_state_dict(legacy)


def test_checkpoint_file_roundtrip(tmp_path):
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': 2})
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=2)
    sched = kfac.KFACParamScheduler(pre, damping_alpha=0.5, damping_schedule=[1])
    run_steps(model, pre, data, 2)
    path = tmp_path / 'ckpt.pt'
    torch.save({'preconditioner': pre.state_dict(), 'schedulers': [sched.state_dict()]}, path)
    blob = torch.load(path, weights_only=False)
    pre.load_state_dict(blob['preconditioner'])
    sched.load_state_dict(blob['schedulers'][0])


def test_mem_opt_inverses_not_saved():
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': 1})
    pre = kfac.KFAC(model, comm_method=kfac.CommMethod.MEM_OPT, factor_update_freq=1,
                    inv_update_freq=1)
    run_steps(model, pre, data, 1)
    with pytest.warns(UserWarning):
        sd = pre.state_dict(include_layer_inverses=True)
    assert all(set(l) == {'A', 'G'} for l in sd['layers'])


def test_param_scheduler():
    pre = kfac.KFAC(SmallNet(), damping=0.01, factor_update_freq=10, inv_update_freq=100)
    s = kfac.KFACParamScheduler(pre, damping_alpha=0.5, damping_schedule=[2, 4],
                                update_freq_alpha=2, update_freq_schedule=[3])
    s.step()  # 1
    assert pre.param_groups[0]['damping'] == 0.01
    s.step()  # 2
    assert pre.param_groups[0]['damping'] == 0.005
    s.step()  # 3
    assert pre.param_groups[0]['factor_update_freq'] == 20
    assert pre.param_groups[0]['inv_update_freq'] == 200
    s.step(10)
    assert pre.param_groups[0]['damping'] == 0.0025
    sd = s.state_dict()
    assert set(sd) == {'damping_base', 'damping_alpha', 'damping_schedule',
                       'factor_update_freq_base', 'inv_update_freq_base', 'update_freq_alpha',
                       'update_freq_schedule', '_step'}
    s2 = kfac.KFACParamScheduler(pre)
    s2.load_state_dict(sd)
    assert s2._step == 10


def test_shared_module_requires_accumulate():
    lm = LSTMModel(20, 8, 8, 1, dropout=0.0, tie_weights=True)
    pre = kfac.KFAC(lm, skip_layers=['embedding', 'linear'])
    with pytest.raises(ValueError):
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            pre.register_shared_module(lm.decoder, lm.encoder)
    pre2 = kfac.KFAC(lm, skip_layers=['embedding', 'linear'], accumulate_data=True)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        pre2.register_shared_module(lm.decoder, lm.encoder, reverse_hooks=True)
    assert len(pre2.layers) == 3


def test_memory_usage_and_repr():
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': 1})
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=1)
    run_steps(model, pre, data, 1)
    assert pre.memory_usage() > 0
    r = repr(pre)
    assert 'registered_layers: 5' in r and 'damping' in r


def test_inplace_relu_after_conv_hooks():
    """Tensor hooks must see the gradient of the conv output, not of the
    in-place ReLU that overwrote it (module full-backward hooks cannot even
    run here: they forbid the in-place op)."""
    torch.manual_seed(0)
    conv = nn.Conv2d(3, 4, 3)
    lin = nn.Linear(4 * 36, 2)
    m = nn.Sequential(conv, nn.ReLU(inplace=True), nn.Flatten(), lin)
    pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=1)
    x = torch.randn(2, 3, 8, 8)
    y = torch.tensor([0, 1])
    nn.functional.cross_entropy(m(x), y).backward()
    out = conv(x)
    out.retain_grad()
    nn.functional.cross_entropy(lin(torch.relu(out).flatten(1)), y).backward()
    assert torch.allclose(pre.layers[0].g_outputs[0], out.grad)


def test_grad_arena_rebinds_after_set_to_none():
    """GradientAllreduce keeps averaging the right tensors when an optimizer's
    zero_grad(set_to_none=True) made backward allocate .grad outside the arena."""
    import torch.nn.functional as F
    from distributed_kfac_pytorch_amd.parallel.grad_sync import GradientAllreduce
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    sync = GradientAllreduce(model)
    assert sync.check_views()
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    opt.zero_grad(set_to_none=True)
    x, y = torch.randn(4, 6), torch.randint(0, 3, (4,))
    F.cross_entropy(model(x), y).backward()
    want = [p.grad.clone() for p in model.parameters()]
    assert not sync.check_views()
    sync()
    assert sync.check_views()
    for (p, view), w in zip(sync.views, want):
        assert p.grad.data_ptr() == view.data_ptr()
        assert torch.equal(p.grad, w)


def test_load_state_dict_keeps_plan_and_buffers():
    """Reloading a checkpoint with unchanged factor shapes keeps the execution
    plan (the arenas a captured graph addresses); the inverses are recomputed."""
    import torch.nn.functional as F
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=2)
    for _ in range(3):
        x, y = torch.randn(4, 6), torch.randint(0, 3, (4,))
        model.zero_grad()
        F.cross_entropy(model(x), y).backward()
        pre.step()
    plan, gen = pre.plan, pre.plan_generation
    qa = pre.layers[0].state['QA']
    pre.load_state_dict(pre.state_dict())
    assert pre.plan is plan and pre.plan_generation == gen
    assert pre.layers[0].state['QA'].data_ptr() == qa.data_ptr()


def test_early_inverse_leading_group_and_cpu_noop():
    """eigen.leading_group names the split solve's first (critical) group --
    every factor above half the largest; the early inverse update needs it
    to hold A factors only and the native GPU path, so on the CPU it is off
    and arming is a no-op (step() solves everything in one batch)."""
    from distributed_kfac_pytorch_amd.ops import eigen
    assert eigen.leading_group([4608, 512, 4608, 2304, 2305, 10]) == [0, 2, 4]
    assert eigen.leading_group([64]) == [0]
    assert eigen.leading_group([]) is None
    m = resnet_cifar.resnet20()
    pre = kfac.KFAC(m, factor_update_freq=1, inv_update_freq=2)
    assert pre.early_inverse is False          # opt-in
    pre.early_inverse = True
    x, y = torch.randn(4, 3, 32, 32), torch.randint(0, 10, (4,))
    for _ in range(3):
        nn.functional.cross_entropy(m(x), y).backward()
        assert pre.arm_early_inverse() is False
        assert pre.disarm_early_inverse() is False
        pre.step()
    assert pre.early_inverse_jobs() == [] and pre.early_inverse_launches == 0
