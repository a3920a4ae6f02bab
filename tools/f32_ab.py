"""A/B timing of the f32 convolutions (the 4^2..16^2 blocks) with pre-split operands (SG2_F32S3) vs the in-loop
split, at the 256^2 Claro network's shapes (bs32; Dmain's batched D runs 64).  HIP-event timing, warm.

    python tools/f32_ab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gan-track_amd'))

import torch  # noqa: E402

from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

DEV = torch.device('cuda', 0)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    shapes = [(64, 512, 16, 512), (32, 512, 16, 512), (32, 512, 8, 512), (64, 512, 8, 512), (32, 512, 4, 512)]
    for N, C, R, O in shapes:
        x = torch.randn(N, C, R, R, device=DEV).contiguous(memory_format=torch.channels_last)
        w = torch.randn(O, C, 3, 3, device=DEV) / (C * 9) ** 0.5
        g = torch.randn(N, O, R, R, device=DEV).contiguous(memory_format=torch.channels_last)
        s = torch.rand(N, C, device=DEV) + 0.5
        d = torch.rand(N, O, device=DEV) + 0.5
        wp = cg._pack_conv(w)
        res = {}
        for p3 in (False, True):
            cg.presplit = p3
            res[p3] = (timeit(lambda: cg.conv_fused(x, wp, O, R, R, 3, 3, 1, (1, 1), in_scale=s, out_scale=d)),
                       timeit(lambda: cg._wgrad_raw(g, x, 3, 3, 1, (1, 1), x_scale=s)),
                       timeit(lambda: cg.split3(x, s)))
        flops = 2 * N * R * R * C * O * 9 / 1e12
        print(f'N{N} C{C} {R}^2 -> {O}: fwd {res[False][0]:.3f} -> {res[True][0]:.3f} ms '
              f'({flops / res[True][0] * 1e3:.0f} TFLOP/s f32), wgrad {res[False][1]:.3f} -> {res[True][1]:.3f} ms, '
              f'split {res[True][2]:.3f} ms', flush=True)


if __name__ == '__main__':
    main()
