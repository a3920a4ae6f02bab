"""Does a captured phase graph replay the same gradient twice (GPU)?  The graph-mode trainer on the Claro 32^2
test network: iteration 0 eager, iteration 1 captures Gmain (then Dmain).  Gmain's graph is replayed again with
the same staged inputs (a) right after its capture, before anything else runs, and (b) after the rest of
iteration 1 (Dmain's capture and replay); G's flat gradient is compared with the first replay's after each.
(The replays also run Gmain's Adam launch and Dmain's updates D: the comparison is of the gradient each replay
writes, with the G and D parameters and G's buffers restored to their values at the first replay.)  Usage: python tools/graph_replay_check.py"""
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden'), os.path.join(ROOT, 'gan-track_amd'), ROOT]
from golden_util import load  # noqa: E402
from parity_train import build_product, CLARO_AUG  # noqa: E402
from training import augment_mi, loss as loss_mod, trainer as trainer_mod  # noqa: E402

dev = torch.device('cuda', 0)
if os.environ.get('SG2_BLAS'):          # 'cublas' (rocBLAS on ROCm) or 'cublaslt' (hipBLASLt)
    torch.backends.cuda.preferred_blas_library(os.environ['SG2_BLAS'])
print('blas library:', torch.backends.cuda.preferred_blas_library(), flush=True)
z = load('train_claro.npz')
cfg, G, D = build_product(z, dev, False)
G_ema = copy.deepcopy(G).eval()
aug = augment_mi.AugmentPipe(run_dir=None, batch_size=cfg['batch'], **CLARO_AUG).train().requires_grad_(False).to(dev)
aug.p.copy_(torch.as_tensor(0.3))
loss = loss_mod.StyleGAN2Loss(device=dev, G=G, D=D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9,
                              pl_weight=2, pl_no_weight_grad=True)
opt = dict(class_name='torch.optim.Adam', lr=0.0025, betas=[0, 0.99], eps=1e-8)
tr = trainer_mod.Trainer(G, D, G_ema, loss, opt, opt, G_reg_interval=2, D_reg_interval=2, batch_size=cfg['batch'],
                         batch_gpu=cfg['batch'], num_gpus=1, rank=0, device=dev, overlap=False, bucket_mb=32)
gen = torch.Generator(device=dev)
gen.manual_seed(5)


def batch():
    real = torch.rand([cfg['batch'], 1, 32, 32], device=dev, generator=gen) * 2 - 1
    c = torch.nn.functional.one_hot(torch.randint(0, 2, [cfg['batch']], device=dev, generator=gen), 2).float()
    gz = torch.randn([4, cfg['batch'], cfg['z_dim']], device=dev, generator=gen)
    return real, c, gz


real, c, gz = batch()
torch.manual_seed(123)
tr.step([real], [c], [[gz[i]] for i in range(4)], [[c] for _ in range(4)])
real, c, gz = batch()
tr.graphs = True
ph = {p.name: p for p in tr.phases}
G0 = [p.detach().clone() for p in list(G.parameters()) + list(D.parameters()) + list(G.buffers())]
flat = ph['Gmain'].exchange.flat


def replay_gmain(tag, ref=None):
    with torch.no_grad():
        for p, q in zip(list(G.parameters()) + list(D.parameters()) + list(G.buffers()), G0):
            p.copy_(q)
    torch.manual_seed(124)
    ph['Gmain'].opt.prepare(flat, ph['Gmain'].exchange.offsets, tr._graphs['Gmain'].part, 'Gmain')
    tr._graphs['Gmain'].graph.replay()
    torch.cuda.synchronize()
    f = flat.clone()
    if ref is not None:
        d = (f - ref).abs()
        print(f'{tag}: |flat - first| max {float(d.max()):.3g}, finite {bool(torch.isfinite(f).all())}', flush=True)
    return f


from torch_utils import misc  # noqa: E402
n_const = len(misc._constant_cache)
torch.manual_seed(124)
tr._serial += 1
tr._graph_phase(ph['Gmain'], [real], [c], [gz[0]], [c])          # capture + first replay
print(f'misc.constant entries created during the Gmain capture: {len(misc._constant_cache) - n_const}', flush=True)
torch.cuda.synchronize()
first = flat.clone()
print(f'first replay: finite {bool(torch.isfinite(first).all())}, |flat| {float(first.norm()):.4g}', flush=True)
replay_gmain('(a) again right after the capture', first)
torch.manual_seed(124)
tr._graph_phase(ph['Dmain'], [real], [c], [gz[2]], [c])          # Dmain capture + replay
torch.cuda.synchronize()
replay_gmain('(b) after Dmain captured and replayed', first)
tr._graph_phase(ph['Dmain'], [real], [c], [gz[2]], [c])          # a second Dmain replay
torch.cuda.synchronize()
replay_gmain('(c) after a second Dmain replay', first)

# (d) new inputs through the trainer's staging path (as iteration 2 does) against an eager evaluation of the same
# phase on the same state and inputs
real2, c2, gz2 = batch()


def restore():
    with torch.no_grad():
        for p, q in zip(list(G.parameters()) + list(D.parameters()) + list(G.buffers()), G0):
            p.copy_(q)


restore()
torch.manual_seed(125)
tr._serial += 1
tr._graph_phase(ph['Gmain'], [real2], [c2], [gz2[0]], [c2])
torch.cuda.synchronize()
graph_flat = flat.clone()
restore()
torch.manual_seed(125)
g = ph['Gmain']
g.opt.zero_grad(set_to_none=True)
g.module.requires_grad_(True)
tr._accumulate(g, [real2], [c2], [gz2[0]], [c2])
g.module.requires_grad_(False)
g.exchange.finish('Gmain', None)
torch.cuda.synchronize()
d = (flat - graph_flat).abs()
print(f'(d) staged new inputs vs eager: |flat_graph - flat_eager| max {float(d.max()):.3g}, graph finite '
      f'{bool(torch.isfinite(graph_flat).all())}, eager |flat| {float(flat.norm()):.4g}, graph |flat| {float(graph_flat.norm()):.4g}', flush=True)
st = tr._graphs['Gmain']
print('   static z equals the new z:', bool(torch.equal(st.inputs[2][0], gz2[0])), flush=True)


def staged_vs_eager(tag, seed):
    real3, c3, gz3 = batch()
    restore()
    torch.manual_seed(seed)
    tr._serial += 1
    tr._graph_phase(ph['Gmain'], [real3], [c3], [gz3[0]], [c3])
    torch.cuda.synchronize()
    gf = flat.clone()
    restore()
    torch.manual_seed(seed)
    g.opt.zero_grad(set_to_none=True)
    g.module.requires_grad_(True)
    tr._accumulate(g, [real3], [c3], [gz3[0]], [c3])
    g.module.requires_grad_(False)
    g.exchange.finish('Gmain', None)
    torch.cuda.synchronize()
    dd = (flat - gf).abs()
    print(f'{tag}: |flat_graph - flat_eager| max {float(dd.max()):.3g}, graph |flat| {float(gf.norm()):.4g}, '
          f'eager |flat| {float(flat.norm()):.4g}', flush=True)


# (e1) the same staged inputs replayed before and after an EMA launch only; (e2) before and after an eager Gmain
real5, c5, gz5 = batch()


def staged_replay(seed):
    restore()
    torch.manual_seed(seed)
    tr._serial += 1
    tr._graph_phase(ph['Gmain'], [real5], [c5], [gz5[0]], [c5])
    torch.cuda.synchronize()
    return flat.clone()


f0 = staged_replay(126)
f1 = staged_replay(126)
print(f'(e0) staged replay twice: max {float((f1 - f0).abs().max()):.3g}', flush=True)
tr.ema(0.9)
torch.cuda.synchronize()
f2 = staged_replay(126)
print(f'(e1) after an EMA launch: max {float((f2 - f0).abs().max()):.3g}', flush=True)
restore()
g.opt.zero_grad(set_to_none=True)
g.module.requires_grad_(True)
tr._accumulate(g, [real5], [c5], [gz5[0]], [c5])
g.module.requires_grad_(False)
g.exchange.finish('Gmain', None)
torch.cuda.synchronize()
f3 = staged_replay(126)
print(f'(e2) after an eager Gmain: max {float((f3 - f0).abs().max()):.3g}', flush=True)

# (e3..e6) which eager work corrupts a later replay: GEMMs only, G forward only, D forward + backward only
f0 = staged_replay(126)
for _ in range(50):
    a = torch.randn(32, 512, device=dev)
    wt = torch.randn(512, 512, device=dev)
    torch.addmm(torch.zeros(512, device=dev), a, wt.t(), beta=1, alpha=0.5)
    torch.addmm(torch.zeros(512, device=dev), a, wt, beta=0, alpha=0.5)
torch.cuda.synchronize()
f1 = staged_replay(126)
print(f'(e3) after eager addmm calls: max {float((f1 - f0).abs().max()):.3g}', flush=True)
f0 = staged_replay(126)
with torch.no_grad():
    torch.manual_seed(1)
    img = G(gz5[0], c5)
torch.cuda.synchronize()
f1 = staged_replay(126)
print(f'(e4) after an eager G forward (no grad): max {float((f1 - f0).abs().max()):.3g}', flush=True)
f0 = staged_replay(126)
x = img.detach().requires_grad_(True)
torch.autograd.grad(D(x, c5).sum(), [x])
torch.cuda.synchronize()
f1 = staged_replay(126)
print(f'(e5) after an eager D forward + input gradient: max {float((f1 - f0).abs().max()):.3g}', flush=True)
f0 = staged_replay(126)
G.requires_grad_(True)
torch.manual_seed(1)
img = G(gz5[0], c5)
torch.autograd.grad(img.square().sum(), [p for p in G.parameters()], allow_unused=True)
G.requires_grad_(False)
torch.cuda.synchronize()
f1 = staged_replay(126)
print(f'(e6) after an eager G forward + parameter gradients: max {float((f1 - f0).abs().max()):.3g}', flush=True)

# (e7..e10) parts of the eager Gmain phase
f0 = staged_replay(126)
torch.manual_seed(1)
img, _ = loss.run_G(gz5[0], c5)
torch.cuda.synchronize()
f1 = staged_replay(126)
print(f'(e7) after an eager loss.run_G (style mixing, no grad): max {float((f1 - f0).abs().max()):.3g}', flush=True)
f0 = staged_replay(126)
torch.manual_seed(1)
x = img.detach().requires_grad_(True)
torch.autograd.grad(loss.run_D(x, c5).sum(), [x])
torch.cuda.synchronize()
f1 = staged_replay(126)
print(f'(e8) after an eager loss.run_D (augment + D) + input gradient: max {float((f1 - f0).abs().max()):.3g}', flush=True)
f0 = staged_replay(126)
G.requires_grad_(True)
g.opt.zero_grad(set_to_none=True)
torch.manual_seed(1)
img, _ = loss.run_G(gz5[0], c5)
img.square().sum().backward()
G.requires_grad_(False)
torch.cuda.synchronize()
f1 = staged_replay(126)
print(f'(e9) after an eager run_G backward into .grad: max {float((f1 - f0).abs().max()):.3g}', flush=True)
f0 = staged_replay(126)
g.exchange.finish('Gmain', None)
torch.cuda.synchronize()
f1 = staged_replay(126)
print(f'(e10) after exchange.finish of those .grad: max {float((f1 - f0).abs().max()):.3g}', flush=True)
