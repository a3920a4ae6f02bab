"""Micro-benchmark of the upfirdn2d FIR kernels on the G/D layer shapes (GPU): GB/s of the
algorithmic traffic (input + output bytes).  Usage: python tools/fir_micro.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import upfirdn2d  # noqa: E402

dev = torch.device('cuda', 0)
f = upfirdn2d.setup_filter([1, 3, 3, 1], device=dev)


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


for res, C in [(256, 64), (128, 128), (64, 256), (32, 512)]:
    for dt in [torch.float16, torch.float32]:
        x = torch.randn(32, C, res + 1, res + 1, device=dev, dtype=dt).contiguous(memory_format=torch.channels_last)
        ms = timeit(lambda: upfirdn2d.upfirdn2d(x, f, padding=1))
        gb = (x.numel() + 32 * C * res * res) * x.element_size() / 1e9
        x2 = torch.randn(32, C, res, res, device=dev, dtype=dt).contiguous(memory_format=torch.channels_last)
        ms2 = timeit(lambda: upfirdn2d.upfirdn2d(x2, f, padding=2))
        ms3 = timeit(lambda: upfirdn2d.upfirdn2d(x2, f, down=2, padding=1))
        gb3 = (x2.numel() * 5 / 4) * x2.element_size() / 1e9
        print(f'{res}^2 C={C} {str(dt)[6:]}: fir(up-layer) {ms:.3f} ms {gb / ms * 1e3:.0f} GB/s | '
              f'pad-fir {ms2:.3f} ms | down2 {ms3:.3f} ms {gb3 / ms3 * 1e3:.0f} GB/s', flush=True)
