"""Does a captured Greg phase (path-length pass: create_graph VJP through the synthesis network, then its
backward) replay the eager Greg gradient?  The 32^2 test network with every random draw fixed (ADA p = 0, no
style mixing, constant noise, a fixed y pattern); pl_mean is restored before every run, so every run sees the same
state and inputs.  Prints the rel L2 of each run's G gradient against the first eager run: eager E2, replays R1
R2, an eager run E3 after the replays, a replay R3 after E3.  Usage: python tools/greg_replay_check.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden'), os.path.join(ROOT, 'gan-track_amd'), ROOT]
from golden_util import load  # noqa: E402
from parity_train import build_product, CLARO_AUG  # noqa: E402
from training import augment_mi, loss as loss_mod  # noqa: E402
from torch_utils.ops import conv2d_gradfix  # noqa: E402

dev = torch.device('cuda', 0)
z = load('train_claro.npz')
cfg, G, D = build_product(z, dev, False)
aug = augment_mi.AugmentPipe(run_dir=None, batch_size=cfg['batch'], **CLARO_AUG).train().requires_grad_(False).to(dev)
aug.p.zero_()
loss = loss_mod.StyleGAN2Loss(device=dev, G=G, D=D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.0,
                              pl_weight=2, pl_no_weight_grad=os.environ.get('PL_NWG', '1') == '1')
loss_mod.torch = type('T', (), {k: getattr(torch, k) for k in dir(torch) if not k.startswith('__')})()
loss_mod.torch.randn_like = lambda t: torch.sin(torch.arange(t.numel(), device=t.device, dtype=t.dtype)).reshape(t.shape)
_fwd = G.synthesis.forward
G.synthesis.forward = lambda ws, **kw: _fwd(ws, **{**kw, 'noise_mode': 'const'})
if os.environ.get('ZB') == '1':     # the beta = 0 GEMM operands zero-filled instead of uninitialised
    from training import networks_stylegan2 as _net
    _net._zero_scalar = lambda t: torch.zeros((), dtype=t.dtype, device=t.device)
    _net._zero_vec = lambda t, n: torch.zeros((n,), dtype=t.dtype, device=t.device)
params = list(G.parameters())
gen = torch.Generator(device=dev)
gen.manual_seed(5)
gz = torch.randn([cfg['batch'], cfg['z_dim']], device=dev, generator=gen)
c = torch.nn.functional.one_hot(torch.randint(0, 2, [cfg['batch']], device=dev, generator=gen), 2).float()
real = torch.rand([cfg['batch'], 1, 32, 32], device=dev, generator=gen) * 2 - 1
pl0 = loss.pl_mean.clone()


def greg():
    G.requires_grad_(True)
    with conv2d_gradfix.pack_cache():
        loss.accumulate_gradients(phase='Greg', real_img=real, real_c=c, gen_z=gz, gen_c=c, gain=2, cur_nimg=0)
    G.requires_grad_(False)


def eager():
    for p in params:
        p.grad = None
    loss.pl_mean.copy_(pl0)
    greg()
    torch.cuda.synchronize()
    return [p.grad.clone() if p.grad is not None else None for p in params], loss.pl_mean.clone()


def rel(a, b):
    num = sum(float((x - y).double().square().sum()) for x, y in zip(a[0], b[0]) if x is not None)
    den = sum(float(x.double().square().sum()) for x in a[0] if x is not None)
    worst = max((float((x - y).abs().max()), i) for i, (x, y) in enumerate(zip(a[0], b[0])) if x is not None)
    names = [n for n, _ in G.named_parameters()]
    return f'rel L2 {(num / max(den, 1e-30)) ** 0.5:.3g}, worst {worst[0]:.3g} ({names[worst[1]]}), pl_mean {float(b[1]):.6g}'


# SNAP=1: every tensor returned by a top-level function of the ops modules is cloned inside the capture; the
# clones of two replays are compared in call order (the first call whose output differs is the culprit)
SNAP = os.environ.get('SNAP') == '1'
REC, snaps = [False], []
if SNAP:
    import inspect
    from torch_utils.ops import modconv, upfirdn2d, bias_act, fma, conv2d_resample
    from training import networks_stylegan2 as _netm

    def _wrap(mod, name, fn):
        def w(*a, **k):
            out = fn(*a, **k)
            if REC[0]:
                outs = out if isinstance(out, (tuple, list)) else (out,)
                for j, t in enumerate(outs):
                    if isinstance(t, torch.Tensor) and t.is_cuda:
                        snaps.append((f'{mod.__name__}.{name}[{j}] {tuple(t.shape)}', t.detach().clone()))
            return out
        return w
    for mod in (conv2d_gradfix, modconv, upfirdn2d, bias_act, fma, conv2d_resample, _netm):
        for name, fn in list(vars(mod).items()):
            if inspect.isfunction(fn) and fn.__module__ == mod.__name__ and not name.startswith('__') and name not in (
                    'pack_cache', 'no_weight_gradients', '_split_k', '_workspace'):
                setattr(mod, name, _wrap(mod, name, fn))
eager()                 # warm-up: lazily created buffers exist before the capture
E1 = eager()
print('E2 (eager again):', rel(E1, eager()), flush=True)
for p in params:
    p.grad = None
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
loss.pl_mean.copy_(pl0)
REC[0] = SNAP
with torch.cuda.graph(g):
    greg()
REC[0] = False
print('snapshots:', len(snaps), flush=True)
held = [p.grad for p in params]
print('grads present after capture:', sum(t is not None for t in held), 'of', len(held), flush=True)


def replay():
    loss.pl_mean.copy_(pl0)
    g.replay()
    torch.cuda.synchronize()
    return [t.clone() if t is not None else None for t in held], loss.pl_mean.clone()


print('R1 (first replay):', rel(E1, replay()), flush=True)
s1 = [t.cpu() for _, t in snaps]
print('R2 (second replay):', rel(E1, replay()), flush=True)
if SNAP:
    shown = 0
    for (name, t), a in zip(snaps, s1):
        b = t.cpu()
        d = float((a.double() - b.double()).abs().max()) if a.numel() else 0.0
        if not d == 0.0:
            print(f'  differs: {name}: max |R2 - R1| {d:.3g} (|R1| max {float(a.double().abs().max()):.3g})', flush=True)
            shown += 1
            if shown >= 12:
                break
    print('  identical snapshots before the first difference:', next((i for i, ((_, t), a) in enumerate(zip(snaps, s1))
          if not float((a.double() - t.cpu().double()).abs().max() if a.numel() else 0) == 0.0), len(snaps)), flush=True)
print('E3 (eager after replays):', rel(E1, eager()), flush=True)
print('R3 (replay after E3):', rel(E1, replay()), flush=True)
