"""A/B of the halo kernel's direct epilogue (SG2_HALO_DIRECT=1, default) against the LDS-transposed one (=0) on the
bench's halo shapes: the modulated synthesis layer with the full epilogue and raw output (G forward), and the dgrad
form with out_scale + dot (G backward).  Prints ms per launch and TFLOP/s.  Usage: python tools/halo_direct_ab.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

dev = torch.device('cuda', 0)
_t = torch.randn(4096, 4096, device=dev, dtype=torch.float16)
for _ in range(200):
    _t = (_t @ _t).clamp_(-1, 1)


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


for N, C, R in [(32, 128, 128), (32, 256, 64), (32, 512, 32), (64, 128, 128), (32, 512, 16)]:
    x = torch.randn(N, C, R, R, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv((torch.randn(C, C, 3, 3, device=dev) / np.sqrt(9 * C)).to(torch.float16))
    s = torch.rand(N, C, device=dev) + 0.5
    nz = torch.randn(N, R, R, device=dev, dtype=torch.float16)
    b = torch.zeros(C, device=dev)
    src = torch.randn(N, C, R, R, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    fl = 2.0 * N * C * C * 9 * R * R
    out = []
    for env in ('0', '1', '0', '1'):
        os.environ['SG2_HALO_DIRECT'] = env
        ms1 = timeit(lambda: cg.conv3x3_fused(x, wp, C, in_scale=s, out_scale=s, noise=nz, noise_gain=0.1, bias=b,
                                              act=1, gain=1.41, clamp=256.0, want_raw=True))
        ms2 = timeit(lambda: cg.conv3x3_fused(x, wp, C, out_scale=s, dot_src=src))
        out.append(f'direct={env}: fwd {ms1:.4f} ms ({fl / ms1 / 1e9:.0f} TF/s) dgrad+dot {ms2:.4f} ms ({fl / ms2 / 1e9:.0f} TF/s)')
    print(f'N={N} C={C} {R}^2: ' + ' | '.join(out), flush=True)
os.environ['SG2_HALO_DIRECT'] = '1'
