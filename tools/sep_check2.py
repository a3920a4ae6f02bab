"""Debug: limited vs full separable up-sampling on the GPU."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import upfirdn2d  # noqa: E402

DEV = torch.device('cuda', 0)
torch.manual_seed(0)
f = torch.randn(12, device=DEV)
x = torch.randn(2, 1, 32, 32, device=DEV)
big = torch.tensor([100000, 100000], dtype=torch.int32, device=DEV)
yf = upfirdn2d.upsample2d(x, f)
h = upfirdn2d._raw(x, f.unsqueeze(0), 2, 1, 1, 1, 6, 5, 0, 0, False, 1.0)
hl = upfirdn2d._raw_lim(x, f.unsqueeze(0), 2, 1, 1, 1, 6, 5, 0, 0, False, 1.0, big)
v = upfirdn2d._raw(h, f.unsqueeze(1), 1, 2, 1, 1, 0, 0, 6, 5, False, 4.0)
vl = upfirdn2d._raw_lim(h, f.unsqueeze(1), 1, 2, 1, 1, 0, 0, 6, 5, False, 4.0, big)
torch.cuda.synchronize()
print('h vs hl', float((h - hl).abs().max()), float(h.abs().max()), float(hl.abs().max()))
print('v vs vl', float((v - vl).abs().max()), float(v.abs().max()), float(vl.abs().max()))
print('yf vs v', float((yf - v).abs().max()))
print(big.tolist())
