"""Bisect which f32 convolution calls of a phase carry a deviation (GPU): the phase-isolated fixture is run with
the f32-input MFMA kernels (SG2_F32_EXACT=1, read per launch) switched on for a range of the phase's f32 conv
calls only, and the error of the watched gradient vs the float64 answer is printed per range, halving the range
that still removes the deviation.

    python tools/exact_bisect.py c2 Greg grad/Greg/synthesis.b256.conv1.noise_strength"""
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')):
    sys.path.insert(0, p)

import torch  # noqa: E402

import config_parity as cp  # noqa: E402
from golden_util import load  # noqa: E402
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

STATE = {'phase': None, 'n': 0, 'lo': 0, 'hi': 0, 'log': None}
WATCH_PHASE = 'Greg'


def _wrap(fn, kind):
    def w(*a, **k):
        x = a[0]
        if STATE['phase'] != WATCH_PHASE or x.dtype != torch.float32:
            return fn(*a, **k)
        i = STATE['n']
        STATE['n'] += 1
        if STATE['log'] is not None:
            site = next((f'{os.path.basename(f.filename)}:{f.lineno}' for f in reversed(traceback.extract_stack()[:-1])
                         if 'conv2d_gradfix' not in f.filename and 'exact_bisect' not in f.filename), '?')
            STATE['log'].append((i, kind, tuple(x.shape), site))
        on = STATE['lo'] <= i < STATE['hi']
        prev = cg.presplit
        if on:
            os.environ['SG2_F32_EXACT'] = '1'
            cg.presplit = False
        try:
            return fn(*a, **k)
        finally:
            if on:
                os.environ.pop('SG2_F32_EXACT', None)
                cg.presplit = prev
    return w


def main():
    global WATCH_PHASE
    tag = sys.argv[1] if len(sys.argv) > 1 else 'c2'
    WATCH_PHASE = sys.argv[2] if len(sys.argv) > 2 else 'Greg'
    keys = sys.argv[3:] or ['grad/Greg/synthesis.b256.conv1.noise_strength', 'grad/Greg/synthesis.b256.conv1.bias']
    cg.conv_fused = _wrap(cg.conv_fused, 'fused')
    cg._conv_raw = _wrap(cg._conv_raw, 'raw')
    cg._wgrad_raw = _wrap(cg._wgrad_raw, 'wgrad')
    from training import loss as L
    orig_acc = L.StyleGAN2Loss.accumulate_gradients

    def acc(self, *a, **k):
        STATE['phase'] = k.get('phase', a[0] if a else None)
        try:
            return orig_acc(self, *a, **k)
        finally:
            STATE['phase'] = None
    L.StyleGAN2Loss.accumulate_gradients = acc
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}_iso.npz'))
    truth = {k[4:]: v for k, v in fix.items() if k.startswith('f64/')}
    dev = torch.device('cuda', 0)

    def run(lo, hi, log=False):
        STATE.update(n=0, lo=lo, hi=hi, log=[] if log else None)
        got, _ = cp.run_product(cfg, inp, tape, dev, aug_p=cfg['aug_p'], isolated=True)
        errs = [max(cp._tensor_errs(got, truth, k)) for k in keys]
        print(f'exact on calls [{lo}, {hi}): ' + ', '.join(f'{k.split("/")[-1]} {e:.3g}' for k, e in zip(keys, errs)),
              flush=True)
        return errs[0], STATE['log']

    base, log = run(0, 0, log=True)
    n = len(log)
    full, _ = run(0, n)
    print(f'{n} f32 conv calls in {WATCH_PHASE}; none exact {base:.3g}, all exact {full:.3g}', flush=True)
    target = base - 0.7 * (base - full)
    lo, hi = 0, n
    while hi - lo > 1:
        mid = (lo + hi) // 2
        a, _ = run(lo, mid)
        b, _ = run(mid, hi)
        if a <= target:
            hi = mid
        elif b <= target:
            lo = mid
        else:
            print('neither half alone removes the deviation: spread over calls', lo, hi, flush=True)
            break
    for i, kind, shape, site in log[lo:hi]:
        print(f'  call {i}: {kind} {shape} {site}')


if __name__ == '__main__':
    main()
