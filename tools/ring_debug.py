"""Where does the ring C=64 kernel (conv3x3_c64r_kernel) disagree with float64?  Prints per-(tile row, tile col,
row in tile, channel half) error fractions for one shape (debug aid)."""
import os
import sys
import numpy as np
import torch
import torch.nn.functional as F
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

DEV = torch.device('cuda', 0)
N, H, W = [int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (4, 256, 256))]
C = 64
torch.manual_seed(5)
x = torch.randn(N, C, H, W)
w = torch.randn(C, C, 3, 3) / np.sqrt(C * 9)
s = torch.rand(N, C) + 0.5
xd = x.to(DEV, torch.float16).contiguous(memory_format=torch.channels_last)
wp = cg._pack_conv(w.to(DEV, torch.float16))
d = torch.rand(N, C) + 0.5
noise = torch.randn(N, 1, H, W)
b = torch.randn(C) * 0.1
modes = sys.argv[4].split(',') if len(sys.argv) > 4 else ['epi_raw', 'epi', 'bias_only', 'demod_only', 'noise_only']
for mode in modes:
    if mode.startswith('epi') or mode.endswith('_only'):
        kw = dict(bias=b.to(DEV), act=1, alpha=0.2, gain=float(np.sqrt(2)), clamp=1.5)
        if mode in ('epi', 'epi_raw', 'demod_only'):
            kw['out_scale'] = d.to(DEV)
        if mode in ('epi', 'epi_raw', 'noise_only'):
            kw.update(noise=noise.to(DEV, torch.float16).reshape(N, H, W).contiguous(), noise_gain=0.3)
        y, raw = cg.conv3x3_fused(xd, wp, C, in_scale=s.to(DEV), want_raw=(mode == 'epi_raw'), **kw)
        xs = (x.to(torch.float16).float() * s[:, :, None, None]).to(torch.float16).double()
        c = F.conv2d(xs, w.to(torch.float16).double(), padding=1)
        z = c * (d[:, :, None, None] if 'out_scale' in kw else 1) + (noise.to(torch.float16).double() * 0.3 if 'noise' in kw else 0) + b[None, :, None, None]
        ref_y = (F.leaky_relu(z, 0.2) * np.sqrt(2)).clamp(-1.5, 1.5)
        torch.cuda.synchronize()
        for nm, out, ref in [('y', y, ref_y)] + ([('raw', raw, c)] if raw is not None else []):
            out = out.double().cpu()
            bad = ((out - ref).abs() > 0.02 * ref.abs() + 0.02)
            print(f'== {mode} {nm}: bad fraction {bad.float().mean():.4f}  zeros {(out == 0).double().mean():.4f}', flush=True)
            bb = bad.reshape(N, 2, 32, H // 8, 8, W // 32, 32).float()
            print(' by sample', bb.mean(dim=(1, 2, 3, 4, 5, 6)).numpy().round(3))
            print(' by channel half', bb.mean(dim=(0, 2, 3, 4, 5, 6)).numpy().round(3))
            print(' by row in tile', bb.mean(dim=(0, 1, 2, 3, 5, 6)).numpy().round(3))
            print(' by tile row', bb.mean(dim=(0, 1, 2, 4, 5, 6)).numpy().round(3))
            print(' by tile col', bb.mean(dim=(0, 1, 2, 3, 4, 6)).numpy().round(3))
        continue
    if mode == 'plain':
        y, raw = cg.conv3x3_fused(xd, wp, C)
        xs = x.to(torch.float16).double()
    elif mode == 'mod':
        y, raw = cg.conv3x3_fused(xd, wp, C, in_scale=s.to(DEV))
        xs = (x.to(torch.float16).float() * s[:, :, None, None]).to(torch.float16).double()
    else:
        y, raw = cg.conv3x3_fused(xd, wp, C, in_scale=s.to(DEV), want_raw=True)
        xs = (x.to(torch.float16).float() * s[:, :, None, None]).to(torch.float16).double()
    torch.cuda.synchronize()
    ref = F.conv2d(xs, w.to(torch.float16).double(), padding=1)
    out = (raw if mode == 'raw' else y).double().cpu()
    bad = ((out - ref).abs() > 0.02 * ref.abs() + 0.02)          # [N, C, H, W]
    print(f'== {mode}: bad fraction {bad.float().mean():.4f}  zeros {(out == 0).double().mean():.4f}', flush=True)
    b = bad.reshape(N, 2, 32, H // 8, 8, W // 32, 32).float()      # n, half, ch, tile row, row in tile, tile col, col
    print(' by sample', b.mean(dim=(1, 2, 3, 4, 5, 6)).numpy().round(3))
    print(' by channel half', b.mean(dim=(0, 2, 3, 4, 5, 6)).numpy().round(3))
    print(' by row in tile', b.mean(dim=(0, 1, 2, 3, 5, 6)).numpy().round(3))
    print(' by tile row', b.mean(dim=(0, 1, 2, 4, 5, 6)).numpy().round(3))
    print(' by tile col', b.mean(dim=(0, 1, 2, 3, 4, 6)).numpy().round(3))
    print(' by col in tile', b.mean(dim=(0, 1, 2, 3, 4, 5)).numpy().round(3))
