"""A/B of the stride-2 / pad-0 3x3 conv: sg2_conv3x3_s2 (halo kernel, 32x4 output tiles) vs the generic
implicit GEMM (sg2_conv2d_fused) on the discriminator's down-2 layers (bias + lrelu + resnet residual) and
the up-2 layers' input gradients (out_scale + dot) of the 256^2 network (GPU).
Usage: python tools/s2_ab.py"""
import os
import sys

import numpy as np
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


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


SHAPES = [(32, 64, 257, 128), (32, 128, 129, 256), (32, 256, 65, 512), (32, 512, 33, 512), (32, 512, 17, 512),
          (32, 256, 33, 512), (32, 128, 65, 256), (32, 64, 129, 128), (16, 128, 257, 256), (8, 64, 513, 128)]
for (n, cin, h, cout) in SHAPES:
    oh = (h - 3) // 2 + 1
    if n * max(cin, cout) * h * h * 2 >= 2 ** 31:
        continue
    x = torch.randn(n, cin, h, h, device=dev).half().contiguous(memory_format=CL)
    wp = cg._pack_conv((torch.randn(cout, cin, 3, 3, device=dev) / np.sqrt(cin * 9)).half())
    b = torch.randn(cout, device=dev) * 0.1
    r = torch.randn(n, cout, oh, oh, device=dev).half().contiguous(memory_format=CL)
    s = torch.rand(n, cout, device=dev) + 0.5
    src = torch.randn(n, cout, oh, oh, device=dev).half().contiguous(memory_format=CL)
    flops = 2.0 * n * oh * oh * cin * cout * 9
    epi = dict(bias=b, act=1, gain=float(np.sqrt(0.5)), clamp=256.0)
    fa = lambda: cg.conv3x3_fused(x, wp, cout, **epi, want_raw=True, stride=2, residual=r, raw_act=True)
    fb = lambda: cg.conv_fused(x, wp, cout, oh, oh, 3, 3, 2, (0, 0), **epi, residual=r, aux_mode=2)
    da = lambda: cg.conv3x3_fused(x, wp, cout, out_scale=s, dot_src=src, stride=2)
    db = lambda: cg.conv_fused(x, wp, cout, oh, oh, 3, 3, 2, (0, 0), out_scale=s, dot_src=src)
    ta, tb, tc, td = timeit(fa), timeit(fb), timeit(da), timeit(db)
    e1 = rel(fa()[0], fb()[0])
    e2 = rel(da()[2], db()[2])
    print(f'N={n} Cin={cin} {h}^2 -> {oh}^2 Cout={cout}: fwd+res s2 {ta:.3f} ms ({flops / ta / 1e9:.0f} TF) | '
          f'generic {tb:.3f} ms ({flops / tb / 1e9:.0f} TF) || scale+dot s2 {tc:.3f} | generic {td:.3f} ms | '
          f'rel diff y {e1:.1e} dot {e2:.1e}', flush=True)
