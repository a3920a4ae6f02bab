"""Run only bench.py's roofline measurement (the dominant conv launch of the 256^2 layer) -- the
short program the HBM-traffic PMC passes profile (tools/gpu_round.sh)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402

# warm the GPU first (a cold GPU makes the first timed launches 15-20 % slow): the bench measures the roofline
# launch after its training steps
a = torch.randn(4096, 4096, device='cuda', dtype=torch.float16)
for _ in range(400):
    a = (a @ a).clamp_(-1, 1)
torch.cuda.synchronize()
print(bench.roofline(torch.device('cuda', 0), 256, 16384, torch.float16), flush=True)
