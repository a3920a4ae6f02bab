"""Run-to-run spread of the f32 whole-iteration parity (GPU): the product iteration of one configuration
twice on the same inputs and random tape; prints whether the two results agree bitwise and the worst
per-phase errors of each against the float64 answer.  Usage: python tools/f32_repeat.py c4"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden'), os.path.join(ROOT, 'gan-track_amd'), ROOT]
import config_parity as cp  # noqa: E402
from golden_util import load  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else 'c4'
dev = torch.device('cuda', 0)
runs = []
for r in range(2):
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}.npz'))
    got, _ = cp.run_product(cfg, inp, tape, dev)
    worst, _ = cp.judge_f32(got, fix, factor=4.0, check=False)
    print(f'run {r}:', {g: (f'{w[0]:.3g}', f'{w[3]:.2f}', w[4]) for g, w in worst.items() if g.startswith('grad/')},
          flush=True)
    runs.append(got)
diff = [k for k in runs[0] if not np.array_equal(np.asarray(runs[0][k]), np.asarray(runs[1][k]))]
print(f'{len(diff)} of {len(runs[0])} entries differ between the runs; e.g. {diff[:6]}')
