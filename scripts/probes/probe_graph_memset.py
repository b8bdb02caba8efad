"""Probe: does a tensor zero_() captured into a hipGraph re-zero on every replay?"""
import torch

dev = torch.device('cuda')
s = torch.cuda.Stream()
for numel, dt in ((1, torch.float64), (1, torch.float32), (256, torch.float32),
                  (66688, torch.float32), (133376, torch.float32), (1 << 20, torch.float32),
                  (25_557_032, torch.float32)):
    t = torch.full((numel,), 5.0, dtype=dt, device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        t.zero_(); t.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        t.zero_()
        t.add_(1)
    res = []
    for r in range(4):
        t.fill_(7.0)
        g.replay()
        torch.cuda.synchronize()
        res.append((float(t.min()), float(t.max())))
    print(numel, dt, res, flush=True)
