"""Lagged inverse updates (KFAC(inverse_lag=L), opt-in): the eigendata of an
inverse step k is computed from the factors as they were at step k and takes
effect at step k+L; with L=0 (the default) the reference's synchronous
schedule (kfac/preconditioner.py:506-510) is unchanged.  CPU path: the solve
runs inline, the storing is deferred exactly as on the GPU."""
import os

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac
from tests import _dist_worker
from tests._oracle_common import build_case, run_steps
from tests.test_distributed import _single, _spawn


def _make(lag, inv_freq=4):
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': 12})
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=inv_freq, lr=0.05,
                    damping=0.003, inverse_lag=lag)
    return model, data, pre


def test_lag_validation():
    model, _ = build_case({'seed': 0, 'batch': 2, 'steps': 1})
    with pytest.raises(ValueError):
        kfac.KFAC(model, inv_update_freq=4, inverse_lag=4)
    with pytest.raises(ValueError):
        kfac.KFAC(model, inv_update_freq=4, inverse_lag=-1)


def test_lag_zero_is_reference_schedule():
    g0, f0 = _run(0, 9)
    g1, f1 = _run(None, 9)
    for a, b in zip(g0, g1):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


def _run(lag, steps):
    model, data = build_case({'seed': 0, 'batch': 6, 'steps': steps})
    kw = {} if lag is None else {'inverse_lag': lag}
    pre = kfac.KFAC(model, factor_update_freq=1, inv_update_freq=4, lr=0.05, damping=0.003,
                    **kw)
    return run_steps(model, pre, data, steps)


def test_lagged_eigendata_timing():
    """Step 4 launches; steps 4, 5 keep the step-0 eigendata; step 6 stores the
    eigendecomposition of the factors of step 4."""
    lag = 2
    model, data, pre = _make(lag)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    layer = pre.layers[0]
    snap_A = None
    q_hist = []
    for i in range(8):
        x, y = data[i]
        opt.zero_grad()
        torch.nn.functional.cross_entropy(model(x), y).backward()
        pre.step()    # factors of step i are updated inside step(), before any launch
        if i == 4:
            snap_A = layer.state['A'].clone()
            assert pre.inverses_in_flight
        q_hist.append(layer.state['QA'].clone())
        opt.step()
    assert torch.equal(q_hist[4], q_hist[3]) and torch.equal(q_hist[5], q_hist[3])
    assert not torch.equal(q_hist[6], q_hist[5])
    d, Q = torch.linalg.eigh(snap_A.float())
    # eigenvectors up to sign: compare the projectors Q diag(d) Q^T
    R = q_hist[6] @ torch.diag(layer.state['dA']) @ q_hist[6].t()
    assert torch.allclose(R, snap_A, atol=1e-5, rtol=1e-4)
    assert torch.allclose(layer.state['dA'], d.clamp(min=0), atol=1e-6, rtol=1e-5)
    assert not pre.inverses_in_flight


def test_lagged_state_dict_roundtrip():
    model, data, pre = _make(2)
    run_steps(model, pre, data, 5)      # step 4 launched, in flight
    assert pre.inverses_in_flight
    sd = pre.state_dict()
    assert sd['param_groups'][0]['step'] == 5
    pre.load_state_dict(sd)              # recomputes inverses synchronously
    assert not pre.inverses_in_flight


@pytest.mark.parametrize('world,method', [(2, 'COMM_OPT'), (2, 'MEM_OPT'), (4, 'HYBRID_OPT')])
def test_lagged_strategy_equivalence(tmp_path, world, method):
    cfg = {'method': method, 'fraction': 0.5, 'steps': 8, 'inv_freq': 3, 'lag': 2}
    ref_grads, ref_factors = _single(cfg)
    _spawn(_dist_worker.kfac_strategy, world, tmp_path, cfg)
    for r in range(world):
        res = torch.load(os.path.join(str(tmp_path), 'rank{}.pt'.format(r)), weights_only=True)
        for step, (gs, rs) in enumerate(zip(res['grads'], ref_grads)):
            for a, b in zip(gs, rs):
                assert torch.equal(a, b), (r, step, (a - b).abs().max().item())


def test_lagged_solve_failure_surfaces_and_resets():
    """A lagged solve over non-finite factors raises the solver's own error
    (not a TypeError at the step that would store it), clears the pending
    update, and training can continue once the factors are finite again."""
    model, data, pre = _make(2)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)

    def step(i):
        x, y = data[i % len(data)]
        opt.zero_grad()
        torch.nn.functional.cross_entropy(model(x), y).backward()
        pre.step()
        opt.step()

    for i in range(4):          # step 0: synchronous inverse; steps 1-3 plain
        step(i)
    layer = pre.layers[0]
    saved = layer.state['A'].clone()
    layer.state['A'].fill_(float('nan'))
    pre.compute_factor_in_hook = True     # keep the poisoned factor through step 4
    with pytest.raises(FloatingPointError):
        step(4)                 # step 4 launches the lagged solve
    assert pre._pending_inv is None
    layer.state['A'].copy_(saved)
    pre.param_groups[0]['step'] = 5
    for i in range(5, 10):
        step(i)
    for p in model.parameters():
        assert torch.isfinite(p).all()
