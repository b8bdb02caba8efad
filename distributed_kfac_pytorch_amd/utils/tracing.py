"""Wall-clock function tracing and device-event phase timing.

`trace/get_trace/print_trace/clear_trace` keep the reference's decorator API
(kfac/utils.py:8-56) with its two defects fixed: `clear_trace` really clears
and `get_trace(max_history)` honours the history window.

`PhaseTimer` is the MI355X addition: HIP events
recorded on the current stream around each K-FAC pipeline phase, resolved
lazily so timing never forces a host sync inside `step()`.
"""
import collections
import os
import time

import torch

__all__ = ['trace', 'get_trace', 'print_trace', 'clear_trace', 'PhaseTimer']

_FUNC_TRACES = collections.defaultdict(list)


def clear_trace():
    _FUNC_TRACES.clear()


def get_trace(max_history=None):
    out = {}
    for name, times in _FUNC_TRACES.items():
        if max_history is not None:
            times = times[-max_history:]
        if times:
            out[name] = sum(times) / len(times)
    return out


def print_trace(max_history=None):
    for name, t in get_trace(max_history).items():
        print('{}: {}'.format(name, t))


def trace(sync=False):
    """Decorator recording the wall time of each call under the function name.

    With `sync=True` a communication barrier brackets the call (and the
    device is synchronised) so the time covers all ranks' work.
    """
    def decorator(func):
        def timed(*args, **kwargs):
            from .. import comm
            if sync:
                _device_sync()
                comm.backend.barrier()
            t0 = time.perf_counter()
            out = func(*args, **kwargs)
            if sync:
                _device_sync()
                comm.backend.barrier()
            _FUNC_TRACES[func.__name__].append(time.perf_counter() - t0)
            return out
        timed.__name__ = func.__name__
        timed.__doc__ = func.__doc__
        return timed
    return decorator


def _device_sync():
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


def _roctx_ok():
    try:
        torch.cuda.nvtx.range_push('kfac/probe')
        torch.cuda.nvtx.range_pop()
        return True
    except Exception:   # a torch build without roctx/nvtx bindings
        return False


class PhaseTimer(object):
    """Accumulates per-phase device time using events on the current stream.

    Usage:
        timer = PhaseTimer(enabled=True)
        with timer('factors'): ...
        timer.summary()  # {'factors': ms_per_call, ...}; syncs once
    On CPU it falls back to perf_counter.
    """

    def __init__(self, enabled=False, ranges=None):
        self.enabled = enabled
        # roctx ranges 'kfac/<phase>' around every phase (torch.cuda.nvtx binds
        # roctx on ROCm): visible to `rocprofv3 --marker-trace` without the
        # timers' events.  KFAC_ROCTX=1 turns them on process-wide.
        if ranges is None:
            ranges = os.environ.get('KFAC_ROCTX', '0') not in ('', '0')
        self.ranges = bool(ranges) and _roctx_ok()
        self._pending = []           # (name, start_event, end_event)
        self._totals = collections.defaultdict(float)
        self._counts = collections.defaultdict(int)

    class _Ctx(object):
        def __init__(self, timer, name):
            self.timer, self.name = timer, name

        def __enter__(self):
            if self.timer.ranges:
                torch.cuda.nvtx.range_push('kfac/' + self.name)
            if not self.timer.enabled:
                return self
            if torch.cuda.is_available() and torch.cuda.is_initialized():
                self.start = torch.cuda.Event(enable_timing=True)
                self.start.record()
            else:
                self.start = time.perf_counter()
            return self

        def __exit__(self, *exc):
            if self.timer.ranges:
                torch.cuda.nvtx.range_pop()
            if not self.timer.enabled:
                return False
            if isinstance(self.start, float):
                self.timer._totals[self.name] += (time.perf_counter() - self.start) * 1e3
                self.timer._counts[self.name] += 1
            else:
                end = torch.cuda.Event(enable_timing=True)
                end.record()
                self.timer._pending.append((self.name, self.start, end))
            return False

    def __call__(self, name):
        return PhaseTimer._Ctx(self, name)

    def _resolve(self):
        if self._pending:
            self._pending[-1][2].synchronize()
            for name, s, e in self._pending:
                self._totals[name] += s.elapsed_time(e)
                self._counts[name] += 1
            self._pending = []

    def summary(self, per_call=False):
        self._resolve()
        if per_call:
            return {k: self._totals[k] / max(1, self._counts[k]) for k in self._totals}
        return dict(self._totals)

    def counts(self):
        self._resolve()
        return dict(self._counts)

    def reset(self):
        self._resolve()
        self._totals.clear()
        self._counts.clear()
