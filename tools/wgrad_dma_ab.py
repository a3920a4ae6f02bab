"""Timing of the stride-1 3x3 weight gradients on the 256^2 network's shapes (GPU), unscaled and with the
modulation scale: run once per SG2_WGRAD_DMA = 0 (register-staged wgrad3x3_kernel), 1 (LDS-DMA kernel for the
unscaled ones), 2 (LDS-DMA kernel for both).  Prints time, TFLOP/s and |dw| (same numbers across modes up to
f32 summation order).  Usage: SG2_WGRAD_DMA=0|1|2 python tools/wgrad_dma_ab.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

dev = torch.device('cuda', 0)
CL = torch.channels_last


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


mode = os.environ.get('SG2_WGRAD_DMA', '1')
x = torch.randn(32, 64, 256, 256, device=dev).half().contiguous(memory_format=CL)   # GPU warm-up
for _ in range(50):
    x.mul_(1.0)
CASES = [(32, 64, 256, 64), (32, 128, 128, 128), (32, 256, 64, 256), (32, 512, 32, 512), (32, 512, 16, 512)]
for scaled in (False, True):
    for (n, a, gh, b) in CASES:
        g = torch.randn(n, a, gh, gh, device=dev).half().contiguous(memory_format=CL)
        x = torch.randn(n, b, gh, gh, device=dev).half().contiguous(memory_format=CL)
        s = (torch.rand(n, b, device=dev) + 0.5) if scaled else None
        flops = 2.0 * n * gh * gh * a * b * 9
        t = timeit(lambda: cg._wgrad_raw(g, x, 3, 3, 1, (1, 1), x_scale=s))
        t = min(t, timeit(lambda: cg._wgrad_raw(g, x, 3, 3, 1, (1, 1), x_scale=s)))
        dw = cg._wgrad_raw(g, x, 3, 3, 1, (1, 1), x_scale=s)
        print(f'DMA={mode} scaled={int(scaled)} N={n} A={a} {gh}^2 B={b}: {t:.4f} ms ({flops / t / 1e9:.0f} TF) '
              f'|dw| {dw.double().norm().item():.6e}', flush=True)
