"""Launches only the stride-2 LDS-DMA implicit GEMM (conv3x3_s2g_kernel) on one D down shape, 20 times -- the short
program the PMC passes profile (tools/gpu_r05o.sh).  Usage: python tools/s2g_only.py [N Cin H Cout]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

N, Cin, H, Cout = [int(v) for v in sys.argv[1:5]] if len(sys.argv) > 4 else (64, 128, 129, 256)
dev = torch.device('cuda', 0)
x = torch.randn(N, Cin, H, H, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
wp = cg._pack_conv((torch.randn(Cout, Cin, 3, 3, device=dev) / np.sqrt(9 * Cin)).to(torch.float16))
b = torch.zeros(Cout, device=dev)
for _ in range(20):
    cg.conv3x3_fused(x, wp, Cout, bias=b, act=1, gain=1.41, clamp=256.0, stride=2)
torch.cuda.synchronize()
print('done', flush=True)
