"""Timing of the small-depth 1x1 kernels of the toRGB / fromRGB layers (GPU): conv1x1_smallk (fromRGB,
Cin = 1), conv1x1_smallo (toRGB, Cout = 1), wgrad1x1_smalla (toRGB weight gradient, A = 1) at 256^2
bs32 / bs64, and wgrad1x1_smallb (fromRGB weight gradient, B = 1), against HBM bytes.
Usage: python tools/small1x1_ab.py"""
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


for n in (32, 64):
    h, c = 256, 64
    x = torch.randn(n, c, h, h, device=dev).half().contiguous(memory_format=CL)
    img = torch.randn(n, 1, h, h, device=dev).half().contiguous(memory_format=CL)
    s = torch.rand(n, c, device=dev) + 0.5
    w_rgb = cg._pack_conv((torch.randn(1, c, 1, 1, device=dev) * 0.1).half())
    w_from = cg._pack_conv((torch.randn(c, 1, 1, 1, device=dev)).half())
    t_o = timeit(lambda: cg.conv_fused(x, w_rgb, 1, h, h, 1, 1, 1, (0, 0), in_scale=s))
    t_k = timeit(lambda: cg.conv_fused(img, w_from, c, h, h, 1, 1, 1, (0, 0), bias=torch.zeros(c, device=dev), act=1,
                                       gain=2 ** 0.5, aux_mode=1))
    t_w = timeit(lambda: cg._wgrad_raw(img, x, 1, 1, 1, (0, 0), x_scale=s))
    t_b = timeit(lambda: cg._wgrad_raw(x, img, 1, 1, 1, (0, 0)))
    bx = x.numel() * 2
    print(f'N={n}: toRGB conv {t_o:.4f} ms ({bx / t_o / 1e6:.0f} GB/s) | fromRGB conv {t_k:.4f} ms '
          f'({(2 * bx + img.numel() * 2) / t_k / 1e6:.0f} GB/s) | toRGB wgrad {t_w:.4f} ms ({bx / t_w / 1e6:.0f} GB/s)'
          f' | fromRGB wgrad {t_b:.4f} ms ({bx / t_b / 1e6:.0f} GB/s)', flush=True)
