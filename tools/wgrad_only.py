"""Launches only the 16-bit 3x3 weight gradient (conv2d_gradfix._wgrad_raw) on one bench shape, 20 times -- the
short program the PMC passes profile.  Usage: python tools/wgrad_only.py [N C R stride]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

N, C, R, S = [int(v) for v in sys.argv[1:5]] if len(sys.argv) > 4 else (64, 128, 128, 1)
dev = torch.device('cuda', 0)
if S == 1:
    g = torch.randn(N, C, R, R, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    x = torch.randn(N, C, R, R, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    for _ in range(20):
        cg._wgrad_raw(g, x, 3, 3, 1, (1, 1))
else:   # the D down layer: g [N, 2C, R, R], x [N, C, 2R + 1, 2R + 1]
    g = torch.randn(N, 2 * C, R, R, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    x = torch.randn(N, C, 2 * R + 1, 2 * R + 1, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    for _ in range(20):
        cg._wgrad_raw(g, x, 3, 3, 2, (0, 0))
torch.cuda.synchronize()
print('done', flush=True)
