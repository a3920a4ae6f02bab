"""Where two runs of the same f32 product iteration first differ (GPU): runs config_parity.run_product twice on a
fixture with forward hooks on every module of G and D and on the loss's augment / D-input steps, recording each
output in call order, and prints the first records whose values differ between the runs (max abs diff, scale).
Usage: python tools/dmain_diverge.py <tag> [phase-filter]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden'), os.path.join(ROOT, 'gan-track_amd'), ROOT]
import config_parity as cp  # noqa: E402
from golden_util import load  # noqa: E402
from training import loss as loss_mod, networks_stylegan2 as net  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else 'c4p0'
dev = torch.device('cuda', 0)
recs = []
cur = []
orig_init = torch.nn.Module.__call__


def rec(name, t):
    if isinstance(t, torch.Tensor) and t.is_floating_point():
        cur.append((name, t.detach().double().cpu()))


def call(self, *a, **k):
    out = orig_init(self, *a, **k)
    rec(type(self).__name__ + ':' + getattr(self, '_dbg_name', ''), out if not isinstance(out, tuple) else out[0])
    return out


torch.nn.Module.__call__ = call
orig_acc = loss_mod.StyleGAN2Loss.accumulate_gradients


def acc(self, phase, *a, **k):
    cur.append(('PHASE ' + phase, torch.zeros(1)))
    for n_, m in list(self.G.named_modules()) + list(self.D.named_modules()):
        m._dbg_name = n_
    r = orig_acc(self, phase, *a, **k)
    for n_, p in list(self.G.named_parameters()) + list(self.D.named_parameters()):
        if p.grad is not None:
            rec('grad ' + phase + ' ' + n_, p.grad)
    return r


loss_mod.StyleGAN2Loss.accumulate_gradients = acc
for r in range(2):
    cur = []
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}.npz'))
    cp.run_product(cfg, inp, tape, dev, aug_p=cfg.get('aug_p', 0.3))
    recs.append(cur)
a, b = recs
print(f'{len(a)} / {len(b)} records')
shown = 0
for (na, ta), (nb, tb) in zip(a, b):
    if na != nb or ta.shape != tb.shape:
        print('structure differs at', na, nb)
        break
    if na.startswith('PHASE'):
        print(na)
        continue
    d = float((ta - tb).abs().max())
    if d > 0:
        print(f'  {na:60s} diff {d:.3g} scale {float(ta.abs().max()):.3g}')
        shown += 1
        if shown > 40:
            break
