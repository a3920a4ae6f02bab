"""Diagnostic: f32 accuracy of the product's SynthesisLayer (fused modulated conv + demod + noise + bias +
lrelu) at real widths against a float64 evaluation of the reference expression; forward and first-order
gradients w.r.t. x, weight, styles (affine) -- to size the error of each primitive at 256^2 / 128^2 / 16^2."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from training import networks_stylegan2 as net  # noqa: E402
from oracle import sg2_oracle as O  # noqa: E402

dev = torch.device('cuda', 0)


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


for (res, cin, cout, up, n) in [(256, 64, 64, 1, 4), (256, 128, 64, 2, 4), (128, 128, 128, 1, 4), (16, 512, 512, 1, 4),
                                (16, 512, 512, 2, 4)]:
    torch.manual_seed(0)
    rin = res // up
    x = torch.randn(n, cin, rin, rin)
    w = torch.randn(cout, cin, 3, 3)
    s = torch.randn(n, cin) * 0.3 + 1
    dy = torch.randn(n, cout, res, res)
    f = O.setup_filter([1, 3, 3, 1]) if up == 2 else None
    outs = []
    for impl in ['hip', 'f64']:
        if impl == 'hip':
            xd = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
            wd = w.to(dev).requires_grad_(True)
            sd = s.to(dev).requires_grad_(True)
            y = net.modulated_conv2d(xd, wd, sd, up=up, padding=1, resample_filter=None if f is None else f.to(dev),
                                     flip_weight=(up == 1), fused_modconv=False)
            g = torch.autograd.grad((y * dy.to(dev)).sum(), [xd, wd, sd])
        else:
            O.REAL = torch.float64
            xd, wd, sd = [t.double().requires_grad_(True) for t in (x, w, s)]
            y = O.modulated_conv2d(xd, wd, sd, up=up, padding=1, resample_filter=None if f is None else f.double(),
                                   flip_weight=(up == 1), fused_modconv=False)
            g = torch.autograd.grad((y * dy.double()).sum(), [xd, wd, sd])
            O.REAL = torch.float32
        outs.append((y, g))
    (y0, g0), (y1, g1) = outs
    print(f'{res}^2 {cin}->{cout} up{up}: y {rel(y0, y1):.2e}  dx {rel(g0[0], g1[0]):.2e}  dw {rel(g0[1], g1[1]):.2e}  '
          f'ds {rel(g0[2], g1[2]):.2e}', flush=True)
