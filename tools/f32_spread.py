"""Run-to-run and process-to-process spread of the f32 whole-iteration product on one config fixture: runs the
product R times in this process, saves each run's summaries (gpurun_out/spread_<tag>_<label>_<r>.npz) and prints,
per phase, the worst tensors against the float64 answer and the largest differences between this process's runs
and any earlier process's saved runs.  Usage: python tools/f32_spread.py <tag> <label> [R]"""
import glob
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden'), os.path.join(ROOT, 'gan-track_amd'), ROOT]
import config_parity as cp  # noqa: E402
from golden_util import load  # noqa: E402

tag, label = sys.argv[1], sys.argv[2]
R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device('cuda', 0)
out = os.path.join(ROOT, 'gpurun_out')
os.makedirs(out, exist_ok=True)
earlier = sorted(glob.glob(os.path.join(out, f'spread_{tag}_*.npz')))
runs = []
for r in range(R):
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}.npz'))
    got, _ = cp.run_product(cfg, inp, tape, dev, aug_p=cfg.get('aug_p', 0.3))
    np.savez(os.path.join(out, f'spread_{tag}_{label}_{r}.npz'), **{k: np.asarray(v) for k, v in got.items()})
    runs.append(got)
truth = {k[4:]: v for k, v in fix.items() if k.startswith('f64/')}


def errs(a, b):
    res = []
    for k in a:
        if k.endswith('/norm') and k in b and k.startswith('grad/'):
            t = k[:-5]
            if t + '/samples' in a and t + '/numel' in b:
                res.append((max(cp._tensor_errs(a, b, t)), t))
    return sorted(res, reverse=True)


for r, got in enumerate(runs):
    print(f'run {r} vs f64, worst:', [(f'{e:.3g}', t) for e, t in errs(got, truth)[:5]], flush=True)
for r in range(1, R):
    print(f'run {r} vs run 0:', [(f'{e:.3g}', t) for e, t in errs(runs[r], runs[0])[:5]], flush=True)
for f in earlier:
    z = dict(np.load(f))
    print(f'run 0 vs {os.path.basename(f)}:', [(f'{e:.3g}', t) for e, t in errs(runs[0], z)[:5]], flush=True)
