"""Is a hipMemsetAsync captured into a HIP graph re-run on every replay?  x is set to 5 eagerly, the graph
memsets it to 0 and adds 1: every replay must leave 1.  Sizes from 32 B to 4 MiB, with and without a
kernel before the memset in the graph.  Usage: python tools/memset_graph_check.py"""
import ctypes

import torch

dev = torch.device('cuda', 0)
hip = ctypes.CDLL('libamdhip64.so')
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemsetAsync.restype = ctypes.c_int

bad = 0
for n in (8, 64, 1024, 1 << 20):
    for pre in (False, True):
        x = torch.full([n], 5.0, device=dev)
        y = torch.zeros([n], device=dev)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            if pre:
                y.add_(1)
            rc = hip.hipMemsetAsync(x.data_ptr(), 0, n * 4, torch.cuda.current_stream().cuda_stream)
            x.add_(1)
        assert rc == 0, rc
        vals = []
        for _ in range(3):
            x.fill_(5.0)
            g.replay()
            torch.cuda.synchronize()
            vals.append(float(x.max()))
        ok = all(v == 1.0 for v in vals)
        bad += not ok
        print(f'{n * 4:8d} B, kernel before: {pre}: after each replay max(x) = {vals} {"ok" if ok else "WRONG"}',
              flush=True)


class _MemsetInBackward(torch.autograd.Function):
    """The memset issued from autograd's backward (its device thread), as the library's accumulators are."""

    @staticmethod
    def forward(ctx, a, buf):
        ctx.buf = buf
        return a * 2

    @staticmethod
    def backward(ctx, g):
        buf = ctx.buf
        rc = hip.hipMemsetAsync(buf.data_ptr(), 0, buf.numel() * 4, torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
        buf.add_(1)
        return g * 2, None


for n in (8, 1 << 20):
    a = torch.ones([4], device=dev, requires_grad=True)
    buf = torch.full([n], 5.0, device=dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        _MemsetInBackward.apply(a, buf).sum().backward()
    vals = []
    for _ in range(3):
        buf.fill_(5.0)
        g.replay()
        torch.cuda.synchronize()
        vals.append(float(buf.max()))
    ok = all(v == 1.0 for v in vals)
    bad += not ok
    print(f'{n * 4:8d} B from backward: after each replay max(buf) = {vals} {"ok" if ok else "WRONG"}', flush=True)
print('memset nodes replay correctly' if bad == 0 else f'{bad} cases wrong', flush=True)
