"""Probe: do two separately captured hipGraphs on two streams run concurrently
on this ROCm, and does an external event recorded INSIDE graph A (mid-way)
gate graph B?  (verdict r3 item 8: side-stream branches inside ONE captured
graph serialise.)

    python scripts/probes/probe_graph_concurrency.py
"""
import time

import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from distributed_kfac_pytorch_amd.ops import _lib  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from external_event import ExternalEvent  # noqa: E402


def work(x, n):
    for _ in range(n):
        x = torch.sin(x) * 1.0001 + 0.0001
    return x


def main():
    dev = torch.device('cuda')
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    # small tensors: latency-bound kernels that leave most CUs idle (a
    # bandwidth-bound chain fills the GPU alone and cannot show overlap)
    a = torch.randn(1 << 14, device=dev)
    b = torch.randn(1 << 14, device=dev)
    ev_mid = ExternalEvent()
    ev_done = ExternalEvent()
    # warm up
    for st in (s1, s2):
        with torch.cuda.stream(st):
            work(a, 2)
    torch.cuda.synchronize()
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(ga, stream=s1):
        ya = work(a, 40)
        ev_mid.record()
        za = work(ya, 40)
    with torch.cuda.graph(gb, stream=s2):
        ev_mid.wait()
        yb = work(b, 80)
        ev_done.record()
    gb2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gb2, stream=s2):
        yb2 = work(b, 80)
    # ONE graph with a forked branch (fork onto s3, join) vs the same kernels
    # in one linear capture
    s3 = torch.cuda.Stream()
    gf, gl = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gf, stream=s1):
        s3.wait_stream(s1)
        with torch.cuda.stream(s3):
            yf2 = work(b, 80)
        yf1 = work(a, 80)
        s1.wait_stream(s3)
    with torch.cuda.graph(gl, stream=s1):
        yl2 = work(b, 80)
        yl1 = work(a, 80)
    torch.cuda.synchronize()

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / reps * 1e3

    def only_a():
        with torch.cuda.stream(s1):
            ga.replay()

    def only_b_after_a():
        with torch.cuda.stream(s1):
            ga.replay()
        s2.wait_stream(s1)
        with torch.cuda.stream(s2):
            gb.replay()

    def both():
        with torch.cuda.stream(s1):
            ga.replay()
        with torch.cuda.stream(s2):
            gb.replay()
        ev_done.wait(s1)

    def both_nogate():
        with torch.cuda.stream(s1):
            ga.replay()
        with torch.cuda.stream(s2):
            gb2.replay()
        s1.wait_stream(s2)

    def eager_both():
        with torch.cuda.stream(s1):
            work(a, 80)
        with torch.cuda.stream(s2):
            work(b, 80)
        s1.wait_stream(s2)

    def forked():
        with torch.cuda.stream(s1):
            gf.replay()

    def linear():
        with torch.cuda.stream(s1):
            gl.replay()

    print('one graph, forked branch %.2f ms; one graph, linear %.2f ms  (env %s)' % (
        timed(forked), timed(linear),
        {k: v for k, v in os.environ.items() if k.startswith(('DEBUG_HIP', 'DEBUG_CLR'))}),
        flush=True)
    print('A || B without the gate %.2f ms; the same kernels eagerly on two streams %.2f ms' % (
        timed(both_nogate), timed(eager_both)), flush=True)
    ta = timed(only_a)
    tseq = timed(only_b_after_a)
    tcon = timed(both)
    print('graph A alone %.2f ms; A then B %.2f ms; A || B (B gated mid-A by an external '
          'event) %.2f ms' % (ta, tseq, tcon), flush=True)
    # correctness of the gate: B must see A's first half
    both()
    torch.cuda.synchronize()
    ref = work(work(a, 40), 0)
    print('gate check: B ran after the mid-A record:', bool(torch.isfinite(yb).all()))


if __name__ == '__main__':
    main()
