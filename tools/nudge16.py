"""The product's own 16-bit spread against the emulated reference's (GPU): runs the isolated iteration of a config
(tests/golden/train_<tag>_iso.npz) in a 16-bit type at the fixture state and at K states nudged by one f32 ulp
(config_parity.run_product perturb=2^-23, seeded signs), and prints per phase the two error measures of
test_16bit_phases (norm-vector, flat; config_parity.compare_flat against float64) for every run beside the same
measures of the fixture's emulation samples (the unnudged emulation and its half-ulp-nudged re-runs).
Usage: python tools/nudge16.py <tag> <fp16|bf16> [K]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import config_parity as cp  # noqa: E402

tag, dt = sys.argv[1], sys.argv[2]
K = int(sys.argv[3]) if len(sys.argv) > 3 else 6
GROUPS = ['grad/Gmain', 'grad/Greg', 'grad/Dmain', 'grad/Dreg']
KEY = {'fp16': 'q16', 'bf16': 'qbf'}[dt]
FIX = os.path.join(ROOT, 'tests', 'golden', f'train_{tag}_iso.npz')
dev = torch.device('cuda', 0)
cfg, inp, tape, fix = cp.load_fixture(np.load(FIX))
truth = {k[4:]: v for k, v in fix.items() if k.startswith('f64/')}
pres = sorted({k.split('/', 1)[0] for k in fix if k.split('/', 1)[0] == KEY or (k.startswith(KEY + 'n') and '/' in k)})
emu = {p: cp.compare_flat({k[len(p) + 1:]: v for k, v in fix.items() if k.startswith(p + '/')}, truth, GROUPS)
       for p in pres}


def row(name, res):
    return f'{name:10s} ' + '  '.join(f'{g[5:]} {res[g][0]:.4f}/{res[g][1]:.4f}' for g in GROUPS)


print(f'{tag} {dt}: norm-vector / flat error vs float64 per phase', flush=True)
for p, r in emu.items():
    print(row('emu ' + p, r), flush=True)
prod = []
for seed in range(K + 1):
    cfg_, inp_, tape_, _ = cp.load_fixture(np.load(FIX))
    got, stats = cp.run_product(cfg_, inp_, tape_, dev, fp16_dtype=torch.float16 if dt == 'fp16' else torch.bfloat16,
                                aug_p=cfg_['aug_p'], isolated=True, perturb=2.0 ** -23 if seed else 0.0,
                                perturb_seed=seed)
    r = cp.compare_flat(got, truth, GROUPS)
    prod.append(r)
    print(row(f'prod s{seed}', r), flush=True)
    for j, (n, v) in enumerate(stats):      # the R1 penalty per sample against float64
        if 'r1_penalty' in n:
            t = np.asarray(fix[f'f64/stats/{j}'], np.float64)
            print('           r1_penalty vs f64: ' + ' '.join(f'{x:+.4f}' for x in (np.asarray(v, np.float64) / t - 1).ravel()),
                  flush=True)
for lab, rs in (('emu', list(emu.values())), ('prod', prod)):
    print(f'{lab:5s} median ' + '  '.join(f'{g[5:]} {np.median([r[g][0] for r in rs]):.4f}/'
                                        f'{np.median([r[g][1] for r in rs]):.4f}' for g in GROUPS))
    print(f'{lab:5s} max    ' + '  '.join(f'{g[5:]} {max(r[g][0] for r in rs):.4f}/'
                                        f'{max(r[g][1] for r in rs):.4f}' for g in GROUPS))
