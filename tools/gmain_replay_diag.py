"""Which state a replayed Gmain graph reads stale (GPU): two trainers (eager, graph) on the Claro 32^2 test
network, iterations 0 and 1 as in tools/graph_diverge.py, then at iteration 2 ONLY the Gmain phase, and the
G flat gradient buffers compared (before any optimiser step of that phase in the eager trainer).  With
RECAPTURE=1 the graph trainer drops its Gmain graph first (a fresh capture at iteration 2).
Usage: [RECAPTURE=1] python tools/gmain_replay_diag.py"""
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
z = load('train_claro.npz')
trs, mods = [], []
for mode in ['eager', 'graph']:
    cfg, G, D = build_product(z, dev, False)
    G_ema = copy.deepcopy(G).eval()
    aug = augment_mi.AugmentPipe(run_dir=None, batch_size=cfg['batch'], **CLARO_AUG).train().requires_grad_(False).to(dev)
    aug.p.copy_(torch.as_tensor(0.3))
    loss = loss_mod.StyleGAN2Loss(device=dev, G=G, D=D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9,
                                  pl_weight=2, pl_no_weight_grad=True)
    opt = dict(class_name='torch.optim.Adam', lr=0.0025, betas=[0, 0.99], eps=1e-8)
    tr = trainer_mod.Trainer(G, D, G_ema, loss, opt, opt, G_reg_interval=2, D_reg_interval=2, batch_size=cfg['batch'],
                             batch_gpu=cfg['batch'], num_gpus=1, rank=0, device=dev, overlap=False, bucket_mb=32)
    trs.append(tr)
    mods.append((G, D, G_ema))
gen = torch.Generator(device=dev)
gen.manual_seed(5)


def batch():
    real = torch.rand([cfg['batch'], 1, 32, 32], device=dev, generator=gen) * 2 - 1
    c = torch.nn.functional.one_hot(torch.randint(0, 2, [cfg['batch']], device=dev, generator=gen), 2).float()
    gz = torch.randn([4, cfg['batch'], cfg['z_dim']], device=dev, generator=gen)
    return real, c, gz


def pdiff(ma, mb):
    return max(float((pa - pb).abs().max()) for pa, pb in zip(ma.parameters(), mb.parameters()))


for it in range(2):
    real, c, gz = batch()
    for k, tr in enumerate(trs):
        if it == 1 and k == 1:
            tr.graphs = True
        torch.manual_seed(123 + it)
        tr.step([real], [c], [[gz[i]] for i in range(4)], [[c] for _ in range(4)])
torch.cuda.synchronize()
print(f'after iteration 1: G diff {pdiff(mods[0][0], mods[1][0]):.3g}  D diff {pdiff(mods[0][1], mods[1][1]):.3g}', flush=True)
ptrs = [[p.data_ptr() for p in m.parameters()] for m in mods[1][:2]]
real, c, gz = batch()
eager, graph = trs
ph_e, ph_g = eager.phases[0], graph.phases[0]
assert ph_e.name == 'Gmain'
if os.environ.get('RECAPTURE') == '1':
    graph._graphs.pop('Gmain')
torch.manual_seed(125)
ph_e.opt.zero_grad(set_to_none=True)
ph_e.module.requires_grad_(True)
eager._accumulate(ph_e, [real], [c], [gz[0]], [c])
ph_e.module.requires_grad_(False)
ph_e.exchange.finish('Gmain', None)
torch.manual_seed(125)
graph._serial += 1
st_part, stepped = graph._graph_phase(ph_g, [real], [c], [gz[0]], [c])
torch.cuda.synchronize()
fe, fg = ph_e.exchange.flat, ph_g.exchange.flat
d = (fe - fg).abs()
print(f'RECAPTURE={os.environ.get("RECAPTURE", "0")}: Gmain flat grad |e - g| max {float(d.max()):.3g} '
      f'rel L2 {float(d.norm() / fe.norm()):.3g}; adam in graph {stepped}', flush=True)
G = mods[1][0]
names = [n for n, _ in G.named_parameters()]
worst = sorted(((float(d[o:o + p.numel()].max()), names[i]) for i, (p, o) in
                enumerate(zip(G.parameters(), ph_g.exchange.offsets))), reverse=True)[:6]
print('   worst params:', worst, flush=True)
print('   param storage moved since iteration 1:',
      [sum(a != b for a, b in zip(old, [p.data_ptr() for p in m.parameters()])) for old, m in zip(ptrs, mods[1][:2])])
