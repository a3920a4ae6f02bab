"""Memory-path microbenchmarks (tools/bench_kernels/membench.hip) at the 256^2 x 64-channel bs32 layer's size:
streaming copy, the ring kernel's half-line stores vs whole-line stores, and its LDS-DMA halo stream (3 slots /
2 slots, pad columns loaded or not).  Prints GB/s of the bytes each pattern moves.
    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/bench_kernels/membench.hip -o tools/bench_kernels/libmembench.so
    python tools/membench.py"""
import ctypes
import os
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, 'bench_kernels', 'libmembench.so'))
dev = torch.device('cuda', 0)
N, H, W = 32, 256, 256
npix = N * H * W
x = torch.randn(npix * 64, device=dev).half()
y = torch.empty_like(x)
sink = torch.zeros(4, device=dev)
st = torch.cuda.current_stream(dev).cuda_stream
P = ctypes.c_void_p


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


B = npix * 128
for rep in range(2):
    ms = timeit(lambda: L.run_copy(P(x.data_ptr()), P(y.data_ptr()), npix * 8, 2048, P(st)))
    print(f'copy (read + write {2 * B / 1e6:.0f} MB): {ms:.4f} ms  {2 * B / ms / 1e6:.0f} GB/s')
    for full in (0, 1):
        ms = timeit(lambda: L.run_store(full, P(y.data_ptr()), npix, 256, P(st)))
        print(f'stores {"whole lines" if full else "half lines (ring epilogue)"} ({B / 1e6:.0f} MB): {ms:.4f} ms  {B / ms / 1e6:.0f} GB/s')
    for kill, nslot in [(0, 3), (1, 3), (1, 2)]:
        ms = timeit(lambda: L.run_halo(kill, nslot, P(x.data_ptr()), N, H, W, P(sink.data_ptr()), 256, P(st)))
        req = (npix // 256) * (50 * 1024 if not kill else 50 * 1024 * 0.85)
        print(f'halo DMA ring nslot={nslot} kill_pad={kill}: {ms:.4f} ms  unique input {B / ms / 1e6:.0f} GB/s, '
              f'requested {req / ms / 1e6:.0f} GB/s')
