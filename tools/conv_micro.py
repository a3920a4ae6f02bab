"""Micro-benchmark of the conv kernels on the 256^2 / 128^2 / 64^2 / 32^2 layer shapes (GPU).
Prints ms and TFLOP/s per kernel.  Usage: python tools/conv_micro.py [--which halo,generic,wgrad]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--which', default='halo,generic,wgrad,convT')
ap.add_argument('--reps', type=int, default=20)
ap.add_argument('--shapes', default='256x64,128x128,64x256,32x512')
ap.add_argument('--dtype', default='float16')
args = ap.parse_args()
dev = torch.device('cuda', 0)
dt = getattr(torch, args.dtype)


def warm_gpu(ms=400):
    """Busy the GPU for ~ms before timing: the first kernels of a fresh process run on a cold GPU (the first
    variant timed was 15-20 % slow, profiles/r02_final_c64p_diag2.log)."""
    a = torch.randn(4096, 4096, device=dev, dtype=torch.float16)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    while True:
        for _ in range(20):
            a = (a @ a).clamp_(-1, 1)
        e1.record()
        e1.synchronize()
        if e0.elapsed_time(e1) > ms:
            return


warm_gpu()


def timeit(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


for sh in args.shapes.split(','):
    res, C = [int(v) for v in sh.split('x')]
    N = 32
    x = torch.randn([N, C, res, res], device=dev, dtype=dt).contiguous(memory_format=torch.channels_last)
    w = (torch.randn([C, C, 3, 3], device=dev) / np.sqrt(C * 9)).to(dt)
    wp = cg._pack_conv(w)
    flops = 2.0 * N * C * C * 9 * res * res
    out = []
    s_ = torch.rand([N, C], device=dev) + 0.5
    if 'halo' in args.which:
        d_ = torch.rand([N, C], device=dev) + 0.5
        nz_ = torch.randn([N, res, res], device=dev, dtype=dt)
        b_ = torch.zeros([C], device=dev)
        ms = timeit(lambda: cg.conv3x3_fused(x, wp, C, in_scale=s_, out_scale=d_, noise=nz_, noise_gain=0.1, bias=b_, act=1, gain=1.41, clamp=256.0), args.reps)
        out.append(f'halo-fused {ms:.3f}ms {flops / ms / 1e9:.0f}TF')
        ms = timeit(lambda: cg.conv3x3_fused(x, wp, C, in_scale=s_, out_scale=d_, noise=nz_, noise_gain=0.1, bias=b_, act=1, gain=1.41, clamp=256.0, want_raw=True), args.reps)
        out.append(f'halo-fused+raw {ms:.3f}ms')
        ms = timeit(lambda: cg.conv3x3_fused(x, wp, C), args.reps)
        out.append(f'halo {ms:.3f}ms {flops / ms / 1e9:.0f}TF')
        ms = timeit(lambda: cg.conv3x3_fused(x, wp, C, in_scale=s_), args.reps)
        out.append(f'halo+mod {ms:.3f}ms')
        ms = timeit(lambda: cg.conv3x3_fused(x, wp, C, out_scale=d_, noise=nz_, noise_gain=0.1, bias=b_, act=1, gain=1.41, clamp=256.0), args.reps)
        out.append(f'halo+epi {ms:.3f}ms')
        ms = timeit(lambda: cg.conv3x3_fused(x, wp, C, out_scale=d_, dot_src=x), args.reps)
        out.append(f'halo+scale+dot {ms:.3f}ms')
        ms = timeit(lambda: cg.conv3x3_fused(x, wp, C, in_scale=s_, out_scale=d_, noise=nz_, noise_gain=0.1, bias=b_, act=1, gain=1.41, clamp=256.0), args.reps)
        out.append(f'halo-fused(again) {ms:.3f}ms')
    if 'generic' in args.which:
        ms = timeit(lambda: cg._conv_raw(x, wp, C, res, res, 3, 3, 1, (1, 1), False), args.reps)
        out.append(f'generic {ms:.3f}ms {flops / ms / 1e9:.0f}TF')
    if 'wgrad' in args.which:
        ms = timeit(lambda: cg._wgrad_raw(x, x, 3, 3, 1, (1, 1)), args.reps)
        out.append(f'wgrad {ms:.3f}ms {flops / ms / 1e9:.0f}TF')
        ms = timeit(lambda: cg._wgrad_raw(x, x, 3, 3, 1, (1, 1), x_scale=s_), args.reps)
        out.append(f'wgrad-scaled {ms:.3f}ms {flops / ms / 1e9:.0f}TF')
    if 'convT' in args.which and res >= 64:
        xh = x[:, :, ::2, ::2].contiguous(memory_format=torch.channels_last)
        wt = w.transpose(0, 1).contiguous()
        f2 = 2.0 * N * C * C * 9 * (res // 2) ** 2
        ms = timeit(lambda: cg._conv_raw(xh, cg._pack_convT(wt), C, res + 1, res + 1, 3, 3, 2, (0, 0), True), args.reps)
        out.append(f'convT-s2 {ms:.3f}ms {f2 / ms / 1e9:.0f}TF')
    print(f'{res}^2 C={C}: ' + ' | '.join(out), flush=True)
