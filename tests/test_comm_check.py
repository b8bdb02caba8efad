"""Single-process checks of the comm-consistency checksums (utils/comm_check.py)."""
import torch

from distributed_kfac_pytorch_amd.utils import comm_check


def test_checksums_detect_transpose_and_nan():
    a = torch.randn(5, 5)
    c = comm_check.checksums([a, a.t().contiguous(), a.clone()])
    assert torch.equal(c[0], c[2])
    assert c[0, 0] == c[1, 0] or abs(float(c[0, 0] - c[1, 0])) < 1e-9   # same plain sum
    assert not torch.equal(c[0], c[1])                                   # weighted sum differs
    b = a.clone()
    b[1, 1] = float('nan')
    cb = comm_check.checksums([b])
    assert torch.isfinite(cb).all()


def test_assert_consistent_single_process_is_noop():
    comm_check.assert_consistent([('x', torch.ones(3))], 'phase')


def test_phase_timer_roctx_ranges_balanced(monkeypatch):
    """PhaseTimer(ranges=True) pushes one 'kfac/<phase>' range per phase and
    pops it on exit, also when the phase raises."""
    from distributed_kfac_pytorch_amd.utils import tracing
    pushed = []
    monkeypatch.setattr(torch.cuda.nvtx, 'range_push', lambda n: pushed.append(n) or 0)
    monkeypatch.setattr(torch.cuda.nvtx, 'range_pop', lambda: pushed.pop() and 0)
    t = tracing.PhaseTimer(enabled=True, ranges=True)
    with t('factors'):
        assert pushed == ['kfac/factors']
    assert pushed == []
    try:
        with t('inverses'):
            raise ValueError('x')
    except ValueError:
        pass
    assert pushed == []
    assert 'factors' in t.summary()
