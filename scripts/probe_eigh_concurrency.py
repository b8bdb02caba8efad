"""Does rocSOLVER eigh overlap across streams / host threads on MI355X?

ResNet-50's 108 factor sizes (B=32); compares serial, 4 side streams (one
host thread), and a host-thread pool with one stream per thread.
"""
import concurrent.futures, json, os, sys, time
import torch

SIZES = [64] * 12 + [128] * 12 + [147] + [256] * 26 + [512] * 19 + [576] * 3 + [1000] + \
        [1024] * 14 + [1152] * 4 + [2048] * 6 + [2049] + [2304] * 6 + [4608] * 3
dev = torch.device('cuda:0')
big = [n for n in SIZES if n > 192]
mats = []
for n in big:
    x = torch.randn(n, n + 64, device=dev)
    mats.append(x @ x.t() / (n + 64))
torch.cuda.synchronize()

def serial():
    for A in mats:
        torch.linalg.eigh(A)
    torch.cuda.synchronize()

def threads(k):
    streams = [torch.cuda.Stream() for _ in range(k)]
    order = sorted(range(len(mats)), key=lambda i: -mats[i].shape[0])
    def work(j):
        s = streams[j]
        with torch.cuda.stream(s):
            for i in order[j::k]:
                torch.linalg.eigh(mats[i])
        s.synchronize()
    with concurrent.futures.ThreadPoolExecutor(k) as ex:
        list(ex.map(work, range(k)))
    torch.cuda.synchronize()

res = {}
for name, fn in [('serial', serial), ('threads4', lambda: threads(4)), ('threads8', lambda: threads(8)),
                 ('threads16', lambda: threads(16))]:
    fn()
    t = time.perf_counter(); fn(); dt = time.perf_counter() - t
    res[name + '_ms'] = dt * 1e3
    print(name, '%.1f ms' % (dt * 1e3), flush=True)
os.makedirs('gpurun_out', exist_ok=True)
json.dump(res, open('gpurun_out/eigh_concurrency.json', 'w'), indent=1)
