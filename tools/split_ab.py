"""Timing of the implicit-GEMM conv / weight-gradient launches whose K split is tuned by
SG2_CONV_SPLIT_WGS / SG2_CWGRAD_WGS (GPU): the f32 low-resolution layers and the 16-bit generic weight
gradients of the 256^2 network (bs32).  Usage: SG2_CWGRAD_WGS=... python tools/split_ab.py"""
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


tag = ' '.join(f'{k}={os.environ[k]}' for k in ('SG2_CONV_SPLIT_WGS', 'SG2_CWGRAD_WGS') if k in os.environ) or 'default'
tot = 0.0
for (dt, n, c, h, o, k) in [(torch.float32, 32, 512, 16, 512, 3), (torch.float32, 32, 512, 8, 512, 3),
                            (torch.float32, 32, 512, 4, 512, 3), (torch.float16, 32, 256, 64, 512, 1),
                            (torch.float16, 32, 64, 128, 128, 1)]:
    x = torch.randn(n, c, h, h, device=dev).to(dt).contiguous(memory_format=CL)
    g = torch.randn(n, o, h, h, device=dev).to(dt).contiguous(memory_format=CL)
    wp = cg._pack_conv((torch.randn(o, c, k, k, device=dev) / np.sqrt(c * k * k)).to(dt))
    p = k // 2
    tf = timeit(lambda: cg.conv_fused(x, wp, o, h, h, k, k, 1, (p, p)))
    tw = timeit(lambda: cg._wgrad_raw(g, x, k, k, 1, (p, p)))
    tot += tf + tw
    print(f'[{tag}] {str(dt)[6:]} N={n} C={c} {h}^2 -> {o} k{k}: fwd {tf:.3f} ms, wgrad {tw:.3f} ms', flush=True)
print(f'[{tag}] total {tot:.3f} ms')
