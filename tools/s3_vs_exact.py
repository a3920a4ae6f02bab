import os, sys
ROOT = '/root/repo'
for p in (ROOT, os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')):
    sys.path.insert(0, p)
import torch
import config_parity as cp
from golden_util import load
from torch_utils.ops import conv2d_gradfix as cg
STATE = {'phase': None, 'n': 0}
orig = cg.conv_fused
def w(*a, **k):
    x = a[0]
    if STATE['phase'] != 'Greg' or x.dtype != torch.float32 or STATE['n'] >= 12:
        return orig(*a, **k)
    i = STATE['n']; STATE['n'] += 1
    args = list(a)
    kk = dict(k)
    if kk.get('dot_out') is not None:
        kk['dot_out'] = None
    r1 = orig(*args, **kk)
    os.environ['SG2_F32_EXACT'] = '1'
    r2 = orig(*args, **kk)
    os.environ.pop('SG2_F32_EXACT')
    torch.cuda.synchronize()
    for j, (p, q) in enumerate(zip(r1, r2)):
        if p is None: continue
        d = (p.double() - q.double()).abs()
        rel = d / (q.double().abs() + 1e-30)
        print(f'call {i} out {j} shape {tuple(p.shape)} maxabs {float(d.max()):.3g} of {float(q.abs().max()):.3g}; '
              f'elem rel>1e-4: {int((rel > 1e-4).sum())}, >1e-2: {int((rel > 1e-2).sum())}, worst rel {float(rel.max()):.3g} at val {float(q.flatten()[rel.argmax()]):.3g}; '
              f'nonfinite {int((~torch.isfinite(p)).sum())}/{int((~torch.isfinite(q)).sum())}; kwargs {sorted(kx for kx, v in k.items() if v is not None)}', flush=True)
    return orig(*a, **k)
cg.conv_fused = w
from training import loss as L
oa = L.StyleGAN2Loss.accumulate_gradients
def acc(self, *a, **k):
    STATE['phase'] = k.get('phase', a[0] if a else None)
    try: return oa(self, *a, **k)
    finally: STATE['phase'] = None
L.StyleGAN2Loss.accumulate_gradients = acc
cfg, inp, tape, fix = cp.load_fixture(load('train_c2_iso.npz'))
cp.run_product(cfg, inp, tape, torch.device('cuda', 0), aug_p=cfg['aug_p'], isolated=True)
