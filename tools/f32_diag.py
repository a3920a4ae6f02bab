"""Diagnostic: where does the product's f32 path (num_fp16_res=0) depart from the float64 oracle at the
C2 width (256^2, cbase 16384)?  Stage-by-stage relative errors, deterministic (noise_mode='const', ADA
at a fixed debug percentile), batch 4."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import config_parity as cp  # noqa: E402
from oracle import sg2_oracle as O  # noqa: E402
from training import networks_stylegan2 as net, augment_mi  # noqa: E402

RES = int(os.environ.get('RES', 256))
cfg = dict(z_dim=512, w_dim=512, img_resolution=RES, channel_base=16384, channel_max=512, map_depth=8, mbstd=4,
           batch=4, c_dim=2, img_channels=1)
dev = torch.device('cuda', 0)
inp = cp.make_inputs(cfg)


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


Gp, Dp = cp._nets(net, cfg, 0)
Gp, Dp = Gp.to(dev), Dp.to(dev)
O.REAL = torch.float64
torch.set_default_dtype(torch.float64)
Go, Do = cp._nets(O, cfg, 4)
aug_o = O.AugmentPipe(**cp.CLARO_AUG).double()
torch.set_default_dtype(torch.float32)
z = torch.from_numpy(inp['z'])
c = torch.from_numpy(inp['c'])
real = torch.from_numpy(inp['real'])

with torch.no_grad():
    ws_p = Gp.mapping(z.to(dev), c.to(dev))
    ws_o = Go.mapping(z.double(), c.double())
    print('mapping ws', rel(ws_p, ws_o))
    img_p = Gp.synthesis(ws_p, noise_mode='const')
    img_o = Go.synthesis(ws_o, noise_mode='const')
    print('synthesis img (const noise)', rel(img_p, img_o))
    img_p2 = Gp.synthesis(ws_o.float().to(dev), noise_mode='const')
    print('synthesis img from the same ws', rel(img_p2, img_o))
    lg_p = Dp(real.to(dev), c.to(dev))
    lg_o = Do(real.double(), c.double())
    print('D logits on reals', rel(lg_p, lg_o), lg_p.flatten()[:4].tolist(), lg_o.flatten()[:4].tolist())
aug_p = augment_mi.AugmentPipe(run_dir=None, batch_size=4, **cp.CLARO_AUG).to(dev)
for pct in [0.1, 0.5, 0.9]:
    with torch.no_grad():
        a_p = aug_p(real.to(dev), False, debug_percentile=pct)
        torch.set_default_dtype(torch.float64)
        a_o = aug_o(real.double(), False, debug_percentile=pct)
        torch.set_default_dtype(torch.float32)
    print(f'ADA pipe debug_percentile={pct}', rel(a_p, a_o))

# first-order D gradients of the logits
Dp.requires_grad_(True)
Do.requires_grad_(True)
lg_p = Dp(real.to(dev), c.to(dev))
torch.nn.functional.softplus(-lg_p).sum().backward()
lg_o = Do(real.double(), c.double())
torch.nn.functional.softplus(-lg_o).sum().backward()
po = dict(Do.named_parameters())
errs = sorted(((rel(p.grad, po[n].grad), n) for n, p in Dp.named_parameters() if p.grad is not None), reverse=True)
print('D first-order grads, worst:', [(f'{e:.2g}', n) for e, n in errs[:6]])
Dp.requires_grad_(False)
Do.requires_grad_(False)

# path-length-style second order through G (const noise)
Gp.requires_grad_(True)
Go.requires_grad_(True)
outs = []
for G, ws, img_dev in [(Gp, ws_p.detach().clone(), dev), (Go, ws_o.detach().clone(), None)]:
    ws = ws.requires_grad_(True)
    img = G.synthesis(ws, noise_mode='const')
    y = torch.from_numpy(np.random.RandomState(3).standard_normal(tuple(img.shape))).to(img.dtype)
    if img_dev is not None:
        y = y.to(img_dev)
    gws, = torch.autograd.grad((img * y).sum(), [ws], create_graph=True)
    L = gws.square().sum(2).mean(1).sqrt().sum()
    L.backward()
    outs.append((gws.detach(), {n: p.grad.detach().clone() for n, p in G.named_parameters() if p.grad is not None}))
print('PL J^T y', rel(outs[0][0], outs[1][0]))
errs = sorted(((rel(outs[0][1][n], outs[1][1][n]), n) for n in outs[1][1] if n in outs[0][1]), reverse=True)
print('PL second-order G grads, worst:', [(f'{e:.2g}', n) for e, n in errs[:10]])

# J^T y with and without create_graph, and per block, to locate the imprecise primitive
Gp.requires_grad_(False)
ws = ws_p.detach().clone().requires_grad_(True)
img = Gp.synthesis(ws, noise_mode='const')
y = torch.from_numpy(np.random.RandomState(3).standard_normal(tuple(img.shape))).float().to(dev)
for cg in [False, True]:
    g, = torch.autograd.grad((img * y).sum(), [ws], create_graph=cg, retain_graph=True)
    print(f'J^T y create_graph={cg}', rel(g, outs[1][0]))
    per = [rel(g[:, i], outs[1][0][:, i]) for i in range(g.shape[1])]
    print('   per ws index', ' '.join(f'{e:.1e}' for e in per))
from torch_utils.ops import conv2d_gradfix  # noqa: E402
with conv2d_gradfix.no_weight_gradients():
    g, = torch.autograd.grad((img * y).sum(), [ws], create_graph=True, retain_graph=True)
print('J^T y create_graph + no_weight_gradients', rel(g, outs[1][0]))

# the oracle itself in f32 (the reference's CPU arithmetic) against f64: the conditioning of J^T y
O.REAL = torch.float32
Go32, _ = cp._nets(O, cfg, 4)
ws = ws_o.detach().float().clone().requires_grad_(True)
img32 = Go32.synthesis(ws, noise_mode='const')
y32 = torch.from_numpy(np.random.RandomState(3).standard_normal(tuple(img32.shape))).float()
g32, = torch.autograd.grad((img32 * y32).sum(), [ws])
print('oracle f32 J^T y vs f64', rel(g32, outs[1][0]))
print('   per ws index', ' '.join(f'{rel(g32[:, i], outs[1][0][:, i]):.1e}' for i in range(g32.shape[1])))
print('product vs oracle f32 J^T y', rel(outs[0][0], g32))
