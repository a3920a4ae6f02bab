"""Calibrate FETCH_SIZE for the persistent C=64 conv's access pattern (MI355X_MICROARCH.md, HBM section:
"other access widths are uncalibrated: calibrate on a known byte count in your own access pattern").
The conv reads each 128-byte pixel line of x as two 64-byte half-lines (one per 32-channel chunk, the
second about a chunk later); the guide's x2 correction is calibrated for 16-byte-per-lane whole-line
streaming reads.  This runs, on the same 268 MB fp16 x of the 256^2 layer:
  (a) x.clone()                 -- whole-line streaming read of exactly |x| bytes (the calibrated case)
  (b) the fused 256^2 layer     -- bench.py's roofline launch
Run (b) also under SG2HIP_LIB=tools/diag_libs/libsg2hip_d3.so (MFMAs and stores compiled out: the
half-line reads alone).  Profile with rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (tools/gpu_round.sh calib)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

dev = torch.device('cuda', 0)
N, C, R = 32, 64, 256
x = torch.randn([N, C, R, R], device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
w = (torch.randn([C, C, 3, 3], device=dev) / np.sqrt(C * 9)).to(torch.float16)
wp = cg._pack_conv(w)
s_ = torch.rand([N, C], device=dev) + 0.5
d_ = torch.rand([N, C], device=dev) + 0.5
nz = torch.randn([N, R, R], device=dev, dtype=torch.float16)
b_ = torch.zeros([C], device=dev)
scratch = torch.empty([1 << 28], device=dev, dtype=torch.uint8)    # 256 MiB: evict x between runs
for _ in range(3):
    scratch.zero_()
    y = x.clone(memory_format=torch.channels_last)
    scratch.zero_()
    cg.conv3x3_fused(x, wp, C, in_scale=s_, out_scale=d_, noise=nz, noise_gain=0.1, bias=b_, act=1, gain=1.41,
                     clamp=256.0)
torch.cuda.synchronize()
print('x bytes', x.numel() * 2, 'lib', os.environ.get('SG2HIP_LIB', 'default'), flush=True)
