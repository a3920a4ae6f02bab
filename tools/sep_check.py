"""1-D FIR passes, quick GPU check: upsample2d / downsample2d (12-tap) and upsample2d_limited vs the oracle."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from oracle import sg2_oracle as O  # noqa: E402
from torch_utils.ops import upfirdn2d  # noqa: E402

DEV = torch.device('cuda', 0)
torch.manual_seed(0)
f = torch.randn(12, dtype=torch.float64)
for shp in [(2, 1, 94, 94), (2, 1, 32, 32), (3, 2, 37, 301)]:
    x = torch.randn(shp, dtype=torch.float64)
    xd = x.float().to(DEV)
    for name, fn, ofn in [('up', lambda t, g: upfirdn2d.upsample2d(t, g), lambda t, g: O.upsample2d(t, g)),
                          ('down', lambda t, g: upfirdn2d.downsample2d(t, g), lambda t, g: O.downsample2d(t, g))]:
        y = fn(xd, f.float().to(DEV)).double().cpu()
        r = ofn(x, f)
        print(shp, name, tuple(y.shape), tuple(r.shape), float((y - r).abs().max()), float(r.abs().max()), flush=True)
    big = torch.tensor([100000, 100000], dtype=torch.int32, device=DEV)
    y = upfirdn2d.upsample2d_limited(xd, f.float().to(DEV), (big, big, big, big)).double().cpu()
    r = O.upsample2d(x, f)
    print(shp, 'limited', float((y - r).abs().max()), flush=True)
