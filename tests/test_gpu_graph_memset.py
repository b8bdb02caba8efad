"""Captured memset nodes are rewritten into fill kernels (csrc/graph_fix.hip).

On this ROCm runtime a memset node of a captured hipGraph does not reliably
clear its target on replay; MIOpen zeroes the accumulation workspace of the
channels_last bf16 weight-gradient convolution it picks for ResNet-50's
layer2.0.conv1 (cudnn.benchmark) with such a memset, so a replayed backward
returned the previous user's bytes (1e30 after a poke, NaN in training:
the round-1 forward/backward graph investigation)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from distributed_kfac_pytorch_amd.ops import _lib

pytestmark = pytest.mark.gpu


def _hip():
    return ctypes.CDLL('libamdhip64.so')


@pytest.mark.parametrize('nbytes,offset', [(4, 0), (4096, 0), (1000003, 0), (12 << 20, 0),
                                           (777, 3), (65536, 8)])
def test_memset_node_rewritten(nbytes, offset):
    hip = _hip()
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t,
                                   ctypes.c_void_p]
    buf = torch.full((nbytes + 64,), 7, dtype=torch.uint8, device='cuda')
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = _lib.new_graph()
    before = dict(_lib.graph_memset_stats)
    with torch.cuda.graph(g, stream=s):
        assert hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr() + offset), 0x5a, nbytes,
                                  ctypes.c_void_p(s.cuda_stream)) == 0
    _lib.finalize_graph(g)
    assert _lib.graph_memset_stats['memsets'] - before['memsets'] == 1
    assert _lib.graph_memset_stats['replaced'] - before['replaced'] == int(_lib.FIX_GRAPH_MEMSETS)
    for _ in range(3):
        buf.fill_(7)
        g.replay()
        torch.cuda.synchronize()
        host = buf.cpu()
        assert (host[offset:offset + nbytes] == 0x5a).all()
        assert (host[:offset] == 7).all() and (host[offset + nbytes:] == 7).all()


def test_graphed_resnet50_step_ignores_stale_memory():
    """Whole-step graph of ResNet-50 (channels_last, bf16 autocast, cudnn.benchmark,
    batch 32, SGD): memory freed and filled with 1e30 between replays must not
    reach the gradients (without the memset rewrite layer2.0.conv1.weight's
    gradient came back ~1e30)."""
    prev = torch.backends.cudnn.benchmark
    torch.backends.cudnn.benchmark = True
    try:
        _stale_memory_case()
    finally:
        # a leaked benchmark=True made every later fp32 model pay MIOpen's
        # find for each new convolution (the ResNet-50 parity test: 12 -> 164 s)
        torch.backends.cudnn.benchmark = prev


def _stale_memory_case():
    from distributed_kfac_pytorch_amd import graphs
    from distributed_kfac_pytorch_amd.models import resnet
    torch.manual_seed(0)
    model = resnet.get_model('resnet50').cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.0125, momentum=0.9)
    g = torch.Generator(device='cuda').manual_seed(0)
    x = torch.randn(32, 3, 224, 224, device='cuda', generator=g).to(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (32,), device='cuda', generator=g)

    def step_fn():
        opt.zero_grad(set_to_none=False)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        return loss

    step = graphs.GraphedTrainStep(step_fn, None, [opt])
    for _ in range(6):
        step()
    assert step.replays > 0
    for _ in range(3):
        junk = [torch.full((n,), 1.2345e30, device='cuda') for n in
                (128, 16384, 1 << 20, 4 << 20, 16 << 20, 64 << 20)]
        del junk
        torch.cuda.synchronize()
        loss = step()
        torch.cuda.synchronize()
        worst = max(float(p.grad.float().abs().max()) for p in model.parameters())
        assert worst < 1e3, worst
        assert torch.isfinite(loss)
