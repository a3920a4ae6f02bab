"""Timing of the stride-2 3x3 weight gradients on the 256^2 network's shapes (GPU): run twice, with
SG2_WGRAD_S2=1 (one all-taps launch, wgrad3x3_s2_kernel) and SG2_WGRAD_S2=0 (four phase launches).
Usage: SG2_WGRAD_S2=0|1 python tools/wgrad_s2_ab.py"""
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


mode = os.environ.get('SG2_WGRAD_S2', '1')
# (N, A = g channels, g size, B = x channels): D down layers (g = conv1 output grad, x = FIR'd input) and
# the up layers' transposed convs (g = layer input, x = FIR-adjoint grad at 2h+1)
CASES = [(32, 128, 128, 64, 2), (32, 256, 64, 128, 2), (32, 512, 32, 256, 2), (32, 512, 16, 512, 2),
         (32, 64, 256, 64, 1), (32, 128, 128, 128, 1), (32, 256, 64, 256, 1), (32, 512, 32, 512, 1)]
for (n, a, gh, b, st) in CASES:
    xh = 2 * gh + 1 if st == 2 else gh
    pad = 0 if st == 2 else 1
    g = torch.randn(n, a, gh, gh, device=dev).half().contiguous(memory_format=CL)
    x = torch.randn(n, b, xh, xh, device=dev).half().contiguous(memory_format=CL)
    flops = 2.0 * n * gh * gh * a * b * 9
    t = timeit(lambda: cg._wgrad_raw(g, x, 3, 3, st, (pad, pad)))
    dw = cg._wgrad_raw(g, x, 3, 3, st, (pad, pad))
    print(f'S2={mode} SWZ={os.environ.get("SG2_WGRAD_SWZ", "0")} stride {st} N={n} A={a} g {gh}^2 B={b} x {xh}^2: {t:.3f} ms ({flops / t / 1e9:.0f} TF) '
          f'|dw| {dw.double().norm().item():.6e}', flush=True)
