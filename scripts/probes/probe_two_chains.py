"""Two chains of small dependent kernels on two streams: does a second
latency-bound launch chain slow the first one down, and by how much per
launch?  (The eigensolver's reduction runs the largest factors' column chain
beside the other factors' chain; `profiles/README.md`, round 5, measures ~0.4 ms
lost per ms of overlap.)

Each chain is N in-place adds on a small tensor, captured into one hipGraph
(no host launch cost) and replayed on its own stream; `grid` sets the
workgroups per kernel (elements / 256 per block).  Reported: ms per chain
alone, both together, and the per-launch time of each.

    python scripts/probes/probe_two_chains.py [N]
"""
import sys

import torch


def chain_graph(x, n, stream):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        for _ in range(3):
            x.add_(1.0)
        torch.cuda.current_stream().synchronize()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(n):
                x.add_(1.0)
    return g


def timed(pairs):
    """pairs: [(graph, stream)], replayed concurrently; ms until all done."""
    cur = torch.cuda.current_stream()
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record(cur)
    ends = []
    for g, s in pairs:
        s.wait_event(e0)
        with torch.cuda.stream(s):
            g.replay()
        e = torch.cuda.Event(enable_timing=True)
        e.record(s)
        ends.append(e)
    torch.cuda.synchronize()
    return [e0.elapsed_time(e) for e in ends]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    dev = torch.device('cuda', 0)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for elems_b in (256, 256 * 1024):            # 1 workgroup / 1024 workgroups per kernel
        a = torch.zeros(256, device=dev)
        b = torch.zeros(elems_b, device=dev)
        ga, gb = chain_graph(a, n, s1), chain_graph(b, n, s2)
        for rep in range(3):
            ta, = timed([(ga, s1)])
            tb, = timed([(gb, s2)])
            both = timed([(ga, s1), (gb, s2)])
        print('chain A (1 wg/kernel) %d launches: alone %.2f ms (%.2f us/launch); chain B (%d wg/kernel) '
              'alone %.2f ms (%.2f us); together A %.2f ms (%.2f us/launch), B %.2f ms (%.2f us)' % (
                  n, ta, 1e3 * ta / n, max(1, elems_b // 256), tb, 1e3 * tb / n,
                  both[0], 1e3 * both[0] / n, both[1], 1e3 * both[1] / n), flush=True)


if __name__ == '__main__':
    main()
