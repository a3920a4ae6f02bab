"""1x1 convolution (the D resnet skip after its FIR) on the implicit-GEMM kernel vs hipBLASLt (torch.addmm on
the NHWC view): forward, input gradient and weight gradient at the 256^2 network's skip shapes (bs 64 = Dmain's
batched pass).  Usage: python tools/skip_ab.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

dev = torch.device('cuda', 0)


def t(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for n, r, ci, co in [(64, 128, 64, 128), (64, 64, 128, 256), (64, 32, 256, 512), (32, 128, 64, 128)]:
    x = torch.randn(n, ci, r, r, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(co, ci, 1, 1, device=dev) / ci ** 0.5).half()
    dy = torch.randn(n, co, r, r, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv(w)
    xf = x.permute(0, 2, 3, 1).reshape(-1, ci)
    dyf = dy.permute(0, 2, 3, 1).reshape(-1, co)
    w2 = w.view(co, ci)
    z = torch.empty((), device=dev, dtype=torch.float16)
    a = t(lambda: cg.conv_fused(x, wp, co, r, r, 1, 1, 1, (0, 0), gain=0.7))
    b = t(lambda: torch.addmm(z, xf, w2.t(), beta=0, alpha=0.7))
    c = t(lambda: cg.conv_fused(dy, cg._pack_convT(w), ci, r, r, 1, 1, 1, (0, 0), transpose=True))
    d = t(lambda: torch.mm(dyf, w2))
    e = t(lambda: cg._wgrad_raw(dy, x, 1, 1, 1, (0, 0)))
    f = t(lambda: torch.mm(dyf.t(), xf))
    print(f'N={n} {r}^2 {ci}->{co}: fwd conv {a:.1f} us / addmm {b:.1f}; dgrad {c:.1f} / mm {d:.1f}; '
          f'wgrad {e:.1f} / mm {f:.1f}', flush=True)
