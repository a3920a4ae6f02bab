"""Do independent branches of a captured HIP graph run concurrently?  Times 2 x K tiny kernels on one
stream vs K on each of two forked streams, with a big matmul alongside in the second case."""
import time
import torch

dev = torch.device('cuda', 0)
K = 200
a = [torch.randn(32, 64, device=dev) for _ in range(4)]
big = torch.randn(8192, 8192, device=dev, dtype=torch.float16)


def chain(t, k):
    for _ in range(k):
        t = t * 1.0001
    return t


def timeit(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


s1 = torch.cuda.Stream()
for name, mode in [('one stream, 2K tiny', 0), ('two streams, K tiny each', 1), ('big GEMM only', 2),
                   ('big GEMM + 2K tiny same stream', 3), ('big GEMM || 2K tiny side stream', 4)]:
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        if mode == 0:
            chain(a[0], 2 * K)
        elif mode == 1:
            s1.wait_stream(cur)
            with torch.cuda.stream(s1):
                chain(a[1], K)
            chain(a[0], K)
            cur.wait_stream(s1)
        elif mode == 2:
            for _ in range(4):
                big @ big
        elif mode == 3:
            for _ in range(4):
                big @ big
            chain(a[0], 2 * K)
        else:
            s1.wait_stream(cur)
            with torch.cuda.stream(s1):
                chain(a[1], 2 * K)
            for _ in range(4):
                big @ big
            cur.wait_stream(s1)
    print(f'{name:36s} {timeit(g):8.3f} ms', flush=True)
