"""A/B of the stride-2 weight gradient: the pipelined 16 x 6 kernel (SG2_WGRAD_S2P=1, default) against the 16 x 8
single-buffered one (=0) on the bench's stride-2 shapes (D down layers, N 64 and 32), alternating order.
Usage: python tools/wgrad_s2p_ab.py"""
import os
import sys

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


for N, C, R in [(64, 64, 128), (32, 64, 128), (64, 128, 64), (32, 128, 64), (64, 256, 32), (64, 512, 16)]:
    Co = min(2 * C, 512)
    g = torch.randn(N, Co, R, R, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    x = torch.randn(N, C, 2 * R + 1, 2 * R + 1, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    fl = 2.0 * N * Co * C * 9 * R * R
    out, ref = [], None
    for env in ('0', '1', '0', '1'):
        os.environ['SG2_WGRAD_S2P'] = env
        dw = cg._wgrad_raw(g, x, 3, 3, 2, (0, 0))
        if ref is None:
            ref = dw.clone()
        d = float((dw - ref).abs().max() / ref.abs().max())
        ms = timeit(lambda: cg._wgrad_raw(g, x, 3, 3, 2, (0, 0)))
        out.append(f's2p={env} {ms:.4f} ms ({fl / ms / 1e9:.0f} TF/s, diff {d:.1e})')
    print(f'N={N} g {Co}x{R}^2 x {C}x{2 * R + 1}^2: ' + ' | '.join(out), flush=True)
os.environ['SG2_WGRAD_S2P'] = '1'
