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
        # the up layer's FIR with its fused epilogue (demod scale, noise, bias, lrelu, clamp, aux = c)
        sc = torch.rand(32, C, device=dev) + 0.5
        nz = torch.randn(32, res, res, device=dev, dtype=dt)
        b = torch.randn(C, device=dev) * 0.1
        ms4 = timeit(lambda: upfirdn2d.fir_fused(x, f, 1, gain=4.0, out_scale=sc, noise=nz, bias=b, act=1,
                                                 act_gain=2 ** 0.5, clamp=256.0, aux_mode=1))
        gb4 = gb + 32 * C * res * res * x.element_size() / 1e9
        print(f'{res}^2 C={C} {str(dt)[6:]}: fir(up-layer) {ms:.3f} ms {gb / ms * 1e3:.0f} GB/s | '
              f'+epilogue {ms4:.3f} ms {gb4 / ms4 * 1e3:.0f} GB/s | '
              f'pad-fir {ms2:.3f} ms | down2 {ms3:.3f} ms {gb3 / ms3 * 1e3:.0f} GB/s', flush=True)
# the up-2 adjoint FIR of the D skips (upfirdn_nhwc_up2)
for res, C in [(128, 64), (64, 128), (32, 256)]:
    x = torch.randn(64, C, res, res, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    ms = timeit(lambda: upfirdn2d.upsample2d(x, f, up=2))
    gb = x.numel() * 5 * 2 / 1e9
    print(f'up2 N=64 {res}^2 C={C} float16: {ms:.3f} ms {gb / ms * 1e3:.0f} GB/s', flush=True)
