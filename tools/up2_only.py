"""Launches only the up-2 transposed conv (conv3x3_up2_kernel, edge split) on one G up shape, 20 times -- the short
program the PMC passes profile (tools/gpu_r05ai.sh).  Usage: python tools/up2_only.py [N Cin H Cout]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

N, Cin, H, Cout = [int(v) for v in sys.argv[1:5]] if len(sys.argv) > 4 else (32, 512, 32, 256)
dev = torch.device('cuda', 0)
x = torch.randn(N, Cin, H, H, device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
wp = cg._pack_conv((torch.randn(Cout, Cin, 3, 3, device=dev) / np.sqrt(9 * Cin)).to(torch.float16))
s = torch.rand(N, Cin, device=dev) + 0.5
assert cg._up2_ok(x, Cout, 2 * H + 1, 2 * H + 1, 3, 3, 2, (0, 0), True)
for _ in range(20):
    cg.conv_fused(x, wp, Cout, 2 * H + 1, 2 * H + 1, 3, 3, 2, (0, 0), transpose=True, in_scale=s)
torch.cuda.synchronize()
print('done', flush=True)
