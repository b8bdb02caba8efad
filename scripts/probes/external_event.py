"""Probe-only helper (moved out of the package, verdict r4 item 5): a HIP
event usable across captured graphs, for scripts/probes/probe_graph_concurrency.py.
Measured and not wired in (profiles/README.md, round 4: the cross-graph gate
costs ~0.4 ms)."""
import torch

from distributed_kfac_pytorch_amd.ops._lib import c_vp, check, lib


class ExternalEvent(object):
    """A HIP event usable ACROSS captured graphs: record() during a capture
    becomes an external event-record node of that graph, wait() during
    another capture an external wait node, so graph B replayed on a second
    stream starts when graph A passes the record point (torch.cuda.Event
    refuses `external=True` on ROCm)."""

    def __init__(self):
        self.handle = lib().kfac_event_create()
        if not self.handle:
            raise RuntimeError('hipEventCreateWithFlags failed')

    def record(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream()
        check(lib().kfac_event_record_external(c_vp(self.handle), c_vp(s.cuda_stream)),
              'kfac_event_record_external')

    def wait(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream()
        check(lib().kfac_stream_wait_external(c_vp(s.cuda_stream), c_vp(self.handle)),
              'kfac_stream_wait_external')

    def __del__(self):
        try:
            if self.handle:
                lib().kfac_event_destroy(c_vp(self.handle))
        except Exception:  # pragma: no cover - interpreter shutdown
            pass
