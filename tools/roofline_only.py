"""Run only bench.py's roofline measurement (the dominant conv launch of the 256^2 layer) -- the
short program the HBM-traffic PMC passes profile (tools/gpu_round.sh)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402

print(bench.roofline(torch.device('cuda', 0), 256, 16384, torch.float16), flush=True)
