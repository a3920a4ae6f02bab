"""A/B of the wide stride-2 down layers (GPU): the LDS-DMA implicit GEMM (sg2_conv3x3_s2 -> conv3x3_s2g_kernel)
against the generic implicit GEMM (sg2_conv2d_fused) and the 32 x 4 halo form (SG2_S2G=0), in the D block's
conv1 form (bias + lrelu + gain + clamp + resnet residual, raw activation kept), on the shapes of the bench step
(tools/conv_census.py).  Prints ms per launch, TFLOP/s and the fraction of the dense 16-bit MFMA peak.
Usage: python tools/s2g_ab.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

PEAK = 2500.0
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


for N, Cin, H, Cout in [(64, 64, 257, 128), (32, 64, 257, 128), (64, 128, 129, 256), (32, 128, 129, 256),
                        (64, 256, 65, 512), (32, 256, 65, 512)]:
    OH = (H - 3) // 2 + 1
    x = torch.randn(N, Cin, H, H, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv((torch.randn(Cout, Cin, 3, 3, device=dev) / np.sqrt(9 * Cin)).to(torch.float16))
    b = torch.randn(Cout, device=dev) * 0.1
    res = torch.randn(N, Cout, OH, OH, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    kw = dict(bias=b, act=1, alpha=0.2, gain=float(np.sqrt(0.5)), clamp=256.0)
    fl = 2.0 * N * OH * OH * Cout * Cin * 9
    out = []
    ys = {}
    for name, env in (('s2g', '1'), ('halo32x4', '0')):
        os.environ['SG2_S2G'] = env
        ys[name] = cg.conv3x3_fused(x, wp, Cout, want_raw=True, stride=2, residual=res, raw_act=True, **kw)[0]
        ms = timeit(lambda: cg.conv3x3_fused(x, wp, Cout, want_raw=True, stride=2, residual=res, raw_act=True, **kw))
        out.append(f'{name} {ms:.4f} ms ({fl / ms / 1e9:.0f} TF/s, {fl / ms / 1e9 / PEAK:.2f})')
    os.environ['SG2_S2G'] = '1'
    ys['generic'] = cg.conv_fused(x, wp, Cout, OH, OH, 3, 3, 2, (0, 0), residual=res, aux_mode=2, **kw)[0]
    ms = timeit(lambda: cg.conv_fused(x, wp, Cout, OH, OH, 3, 3, 2, (0, 0), residual=res, aux_mode=2, **kw))
    out.append(f'generic {ms:.4f} ms ({fl / ms / 1e9:.0f} TF/s, {fl / ms / 1e9 / PEAK:.2f})')
    d = (ys['s2g'].float() - ys['generic'].float()).abs().max().item()
    print(f'N={N} Cin={Cin} {H}^2 -> {OH}^2 Cout={Cout}: ' + ' | '.join(out) + f' | max|s2g-generic| {d:.3g}',
          flush=True)
