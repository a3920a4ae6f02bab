"""The f32 (split-bf16) implicit-GEMM convs of the low-resolution blocks (GPU): forward 3x3 and the up
layers' transposed 3x3 at 4^2 / 8^2 / 16^2, bs32 and bs64, timed with the process's SG2_CONV_SPLIT_WGS
(read once per process) and, in the same process, in deterministic mode (split-K partials to slots +
an ordered sum instead of float atomics).  Prints ms and the fraction of the six-product bf16 MFMA peak
(2.5 PFLOP/s dense).  Usage: SG2_CONV_SPLIT_WGS=... python tools/f32_small_ab.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import sg2hip  # noqa: E402
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

dev = torch.device('cuda', 0)
CL = torch.channels_last
PEAK = 2.5e15


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


tag = os.environ.get('SG2_CONV_SPLIT_WGS', 'default(512)')
tot = {False: 0.0, True: 0.0}
for n in (32, 64):
    for h in (4, 8, 16):
        x = torch.randn(n, 512, h, h, device=dev).contiguous(memory_format=CL)
        s = torch.rand(n, 512, device=dev) + 0.5
        wp = cg._pack_conv(torch.randn(512, 512, 3, 3, device=dev) / np.sqrt(512 * 9))
        cases = [('fwd', lambda: cg.conv_fused(x, wp, 512, h, h, 3, 3, 1, (1, 1), in_scale=s)),
                 ('up2T', lambda: cg.conv_fused(x, wp, 512, 2 * h + 1, 2 * h + 1, 3, 3, 2, (0, 0), transpose=True,
                                                in_scale=s))]
        for name, fn in cases:
            flops = 6 * 2.0 * n * h * h * 512 * 512 * 9
            t = {}
            for det in (False, True):
                if det:
                    with sg2hip.deterministic(True, scratch_mb=512, device=dev):
                        t[det] = timeit(fn)
                else:
                    t[det] = timeit(fn)
                tot[det] += t[det]
            print(f'[{tag}] {name} N={n} {h}^2: atomics {t[False]:.3f} ms ({flops / t[False] * 1e3 / PEAK:.0%} of S3 peak) | '
                  f'slots {t[True]:.3f} ms ({flops / t[True] * 1e3 / PEAK:.0%})', flush=True)
print(f'[{tag}] total atomics {tot[False]:.3f} ms, slots {tot[True]:.3f} ms')
