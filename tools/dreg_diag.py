"""Localises a 16-bit Dreg gradient-scale offset (GPU): runs the isolated C2 iteration (tests/config_parity.py,
fixture train_c2_iso.npz) with the product in f32, fp16 and bf16 and, for each, records the gradient arriving at
every discriminator block's output during the Dreg phase's R1 VJP (the first-order backward, create_graph) and
the R1 penalty per sample.  Prints, per block, each 16-bit run's scale against the f32 run
(<g16, g32> / |g32|^2 - 1, the common-mode part) and its relative residual, and the penalty against float64.
Usage: python tools/dreg_diag.py [tag]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import config_parity as cp  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else 'c2'
dev = torch.device('cuda', 0)
FIX = os.path.join(ROOT, 'tests', 'golden', f'train_{tag}_iso.npz')
cfg, inp, tape, fix = cp.load_fixture(np.load(FIX))
names, _ = cp.fixture_stats(fix)

rec = []
orig_nets = cp._nets


def hooked_nets(mod, cfg_, num_fp16_res, fp16_dtype=None, **extra):
    G, D = orig_nets(mod, cfg_, num_fp16_res, fp16_dtype, **extra)
    for name, m in D.named_children():
        if not (name.startswith('b') or name == 'mapping'):
            continue

        def fwd_hook(mod_, args, out, name=name):
            t = out[0] if isinstance(out, tuple) else out
            if torch.is_tensor(t) and t.requires_grad:
                t.register_hook(lambda g, name=name: rec.append((name, g.detach().float().clone())))
        m.register_forward_hook(fwd_hook)
    return G, D


cp._nets = hooked_nets
runs = {}
for dt in ['f32', 'fp16', 'bf16']:
    rec.clear()
    fp = None if dt == 'f32' else (torch.float16 if dt == 'fp16' else torch.bfloat16)
    cfg_, inp_, tape_, fix_ = cp.load_fixture(np.load(FIX))
    got, stats = cp.run_product(cfg_, inp_, tape_, dev, fp16_dtype=fp, aug_p=cfg_['aug_p'], isolated=True)
    runs[dt] = (list(rec), stats)
    print(dt, 'hook firings', len(rec), flush=True)

f32r = runs['f32'][0]
for dt in ['fp16', 'bf16']:
    r = runs[dt][0]
    print(f'== {dt}: {len(r)} firings (f32 {len(f32r)})')
    if len(r) != len(f32r):
        print('   firing counts differ; comparing the common prefix')
    for i, ((n, g), (n32, g32)) in enumerate(zip(r, f32r)):
        if n != n32 or g.shape != g32.shape:
            print(f'   firing {i}: {n} vs {n32} shape {tuple(g.shape)} vs {tuple(g32.shape)} -- stop')
            break
        a, b = g.double().flatten(), g32.double().flatten()
        nb2 = float(b @ b)
        if nb2 == 0:
            continue
        scale = float(a @ b) / nb2 - 1
        resid = float((a - (1 + scale) * b).norm() / b.norm())
        # per-sample scale
        ps = [float(g[k].double().flatten() @ g32[k].double().flatten()) / max(float(g32[k].double().flatten().square().sum()), 1e-300) - 1
              for k in range(g.shape[0])]
        print(f'   {i:3d} {n:10s} {str(tuple(g.shape)):22s} scale {scale:+.5f} resid {resid:.4f} per-sample ' +
              ' '.join(f'{x:+.4f}' for x in ps))

for dt in ['f32', 'fp16', 'bf16']:
    stats = runs[dt][1]
    for j, (n, v) in enumerate(stats):
        if 'r1' in n or 'D/reg' in n or 'scores/real' in n:
            t = np.asarray(fix[f'f64/stats/{j}'], np.float64)
            v = np.asarray(v, np.float64)
            print(f'{dt} stat {j} {n}: rel to f64 ' + ' '.join(f'{x:+.5f}' for x in (v / t - 1).ravel()))
