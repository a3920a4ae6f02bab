"""Diagnostic: per-tensor errors of the product's C1 iteration (f32) against the reference fixture."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import config_parity as cp  # noqa: E402
from golden_util import load  # noqa: E402

z = load('train_c1.npz')
cfg, inp, tape = cp.load_fixture(z)
got, _ = cp.run_product(cfg, inp, tape, torch.device('cuda', 0))
for ph in cp.PHASES:
    keys = sorted(k[:-5] for k in z.files if k.startswith(f'grad/{ph}/') and k.endswith('/norm'))
    tot = np.sqrt(sum(float(z[k + '/norm']) ** 2 for k in keys))
    rows = []
    for k in keys:
        if k + '/norm' not in got:
            continue
        nw, ng = float(z[k + '/norm']), float(got[k + '/norm'])
        rows.append((abs(ng - nw) / max(nw, 1e-30), k, nw, nw / tot))
    rows.sort(reverse=True)
    print(f'== {ph}: total norm {tot:.4g}')
    for e, k, nw, fr in rows[:6]:
        print(f'   {e:.3g}  {k}  norm {nw:.4g}  ({fr:.2g} of phase)')
