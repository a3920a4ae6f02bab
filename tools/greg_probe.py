"""Record the tensors around one synthesis layer's path-length second backward (GPU): the layer's forward output,
the gradient reaching it in the penalty's backward and the layer_bwd results, on a phase-isolated fixture.
Run once per build variant (e.g. SG2_F32_EXACT=0 / 1) and compare the saved files:

    python tools/greg_probe.py save c2 gpurun_out/probe_s3.pt
    SG2_F32_EXACT=1 python tools/greg_probe.py save c2 gpurun_out/probe_exact.pt
    python tools/greg_probe.py cmp gpurun_out/probe_s3.pt gpurun_out/probe_exact.pt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')):
    sys.path.insert(0, p)

import torch  # noqa: E402


def save(tag, out, res=256, cout=64):
    import config_parity as cp
    from golden_util import load
    from torch_utils.ops import conv2d_gradfix as cg, modconv
    rec = {}
    phase = {'name': None}
    orig_lb = cg.layer_bwd
    orig_fc = modconv.FusedConv.forward

    def lb(dy, y, *a, **k):
        r = orig_lb(dy, y, *a, **k)
        if phase['name'] == 'Greg' and tuple(y.shape[1:]) == (cout, res, res):
            i = sum(1 for kk in rec if kk.startswith('lb'))
            rec[f'lb{i}_dy'] = dy.detach().float().cpu()
            rec[f'lb{i}_y'] = y.detach().float().cpu()
            rec[f'lb{i}_dn'] = r[3].detach().float().cpu() if r[3] is not None else None
        return r

    def fc(ctx, x, styles, weight, *a):
        y = orig_fc(ctx, x, styles, weight, *a)
        if phase['name'] == 'Greg' and tuple(y.shape[1:]) == (cout, res, res):
            i = sum(1 for kk in rec if kk.startswith('fwd'))
            rec[f'fwd{i}_y'] = y.detach().float().cpu()
            rec[f'fwd{i}_x'] = x.detach().float().cpu()
            rec[f'fwd{i}_s'] = styles.detach().float().cpu()
        return y
    from training import loss as L
    orig_acc = L.StyleGAN2Loss.accumulate_gradients

    def acc(self, *a, **k):
        phase['name'] = k.get('phase', a[0] if a else None)
        try:
            return orig_acc(self, *a, **k)
        finally:
            phase['name'] = None
    cg.layer_bwd = lb
    modconv.cg_layer_bwd = lb
    modconv._cg.layer_bwd = lb
    modconv.FusedConv.forward = staticmethod(fc)
    L.StyleGAN2Loss.accumulate_gradients = acc
    try:
        cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}_iso.npz'))
        cp.run_product(cfg, inp, tape, torch.device('cuda', 0), aug_p=cfg['aug_p'], isolated=True)
    finally:
        cg.layer_bwd = orig_lb
        modconv.FusedConv.forward = staticmethod(orig_fc)
        L.StyleGAN2Loss.accumulate_gradients = orig_acc
    torch.save(rec, out)
    print('saved', sorted(rec))


def cmp(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    for k in sorted(A):
        if A[k] is None or k not in B or B[k] is None:
            continue
        diff = A[k].double() - B[k].double()
        d = diff.norm() / max(B[k].double().norm(), 1e-300)
        # where the difference lives: share of its energy in the 16 / 256 largest pixels (summed over channels)
        e = (diff ** 2).sum(1).flatten() if diff.ndim == 4 else (diff ** 2).flatten()
        top = torch.sort(e, descending=True).values
        tot = max(float(e.sum()), 1e-300)
        print(f'{k:12s} {tuple(A[k].shape)} rel diff {float(d):.3g}  max abs {float(diff.abs().max()):.3g}  '
              f'energy in top 16 px {float(top[:16].sum()) / tot:.2f}, top 256 {float(top[:256].sum()) / tot:.2f}')
        if diff.ndim == 4 and k.endswith('_dy') and float(d) > 1e-5:
            yk = k[:-3] + '_y'
            for flat in torch.argsort(e, descending=True)[:3].tolist():
                n_, rem = divmod(flat, diff.shape[2] * diff.shape[3])
                yy, xx = divmod(rem, diff.shape[3])
                ya, yb = A[yk][n_, :, yy, xx].double(), B[yk][n_, :, yy, xx].double()
                c = int(torch.argmax(diff[n_, :, yy, xx].abs()))
                print(f'    px (n{n_}, {yy}, {xx}) ch {c}: dy {float(A[k][n_, c, yy, xx]):.4g} / {float(B[k][n_, c, yy, xx]):.4g}'
                      f'  y {float(ya[c]):.4g} / {float(yb[c]):.4g}; min |y| over ch {float(ya.abs().min()):.3g} / '
                      f'{float(yb.abs().min()):.3g}; sign flips {int(((ya > 0) != (yb > 0)).sum())}')


if __name__ == '__main__':
    if sys.argv[1] == 'save':
        save(sys.argv[2], sys.argv[3])
    else:
        cmp(sys.argv[2], sys.argv[3])
