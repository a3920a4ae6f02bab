"""Path-length (Greg) pass: product (GPU, deterministic f32) vs the float64 oracle (CPU), on a phase-isolated
fixture.  Records J^T y per ws row, the path lengths and selected parameter gradients of both sides, and prints
their relative differences -- to localise a Greg gradient that is off while the rest of the phase agrees.

    python tools/greg_diff.py c2 [param-substring ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import config_parity as cp  # noqa: E402
from golden_util import load  # noqa: E402

_rec = {}
_orig_grad = torch.autograd.grad


def _grad(outputs, inputs, *a, **k):
    res = _orig_grad(outputs, inputs, *a, **k)
    ins = inputs if isinstance(inputs, (list, tuple)) else [inputs]
    if len(ins) == 1 and ins[0].ndim == 3 and ins[0].shape[-1] == 512 and 'jty' not in _rec:
        _rec['jty'] = res[0].detach().double().cpu().clone()
    return res


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def run(side, tag, keys):
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}_iso.npz'))
    _rec.clear()
    grads = {}
    torch.autograd.grad = _grad
    try:
        if side == 'product':
            from training import loss as L

            orig_acc = L.StyleGAN2Loss.accumulate_gradients

            def acc(self, phase, *a, **k):
                out = orig_acc(self, phase, *a, **k)
                if phase == 'Greg':
                    for n, p in self.G.named_parameters():
                        if p.grad is not None and any(s in n for s in keys):
                            grads[n] = p.grad.detach().double().cpu().clone()
                return out
            L.StyleGAN2Loss.accumulate_gradients = acc
            try:
                cp.run_product(cfg, inp, tape, torch.device('cuda', 0), aug_p=cfg['aug_p'], isolated=True)
            finally:
                L.StyleGAN2Loss.accumulate_gradients = orig_acc
        else:
            from oracle import sg2_oracle as O
            orig_acc = O.StyleGAN2Loss.accumulate_gradients

            def acc(self, phase, *a, **k):
                out = orig_acc(self, phase, *a, **k)
                if phase == 'Greg':
                    for n, p in self.G.named_parameters():
                        if p.grad is not None and any(s in n for s in keys):
                            grads[n] = p.grad.detach().double().cpu().clone()
                return out
            O.StyleGAN2Loss.accumulate_gradients = acc
            try:
                cp.run_oracle_f64(cfg, inp, tape, cfg['aug_p'], isolated=True)
            finally:
                O.StyleGAN2Loss.accumulate_gradients = orig_acc
    finally:
        torch.autograd.grad = _orig_grad
    return dict(_rec), grads


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else 'c2'
    keys = sys.argv[2:] or ['b256.conv1', 'b256.torgb', 'b256.conv0']
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    rp, gp = run('product', tag, keys)
    ro, go = run('oracle', tag, keys)
    jp, jo = rp['jty'].numpy(), ro['jty'].numpy()
    print('J^T y rows rel diff:', [round(_rel(jp[:, i], jo[:, i]), 7) for i in range(jp.shape[1])])
    lp, lo = np.sqrt((jp ** 2).sum(2).mean(1)), np.sqrt((jo ** 2).sum(2).mean(1))
    print('pl lengths product', lp, 'oracle', lo)
    for n in sorted(go):
        if n in gp:
            print(f'{n:50s} rel {_rel(gp[n].numpy(), go[n].numpy()):.4g}  |oracle| {np.linalg.norm(go[n].numpy()):.4g}'
                  f'  |product| {np.linalg.norm(gp[n].numpy()):.4g}')
        else:
            print(f'{n:50s} missing in product')


if __name__ == '__main__':
    main()
