"""Eager vs HIP-graph training, iteration by iteration (GPU): the Claro 32^2 test network, reg intervals 2, the
same inputs; prints after every iteration the largest parameter difference between the two trainers and where.
Usage: python tools/graph_diverge.py [iterations] [num_gpus_simulated] [graph|eager: the second trainer's mode]"""
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.environ.get('SG2_PKG_ROOT', ROOT)     # (bisection: an older tree of the package, same tests)
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden'), os.path.join(PKG, 'gan-track_amd'), ROOT]
from golden_util import load  # noqa: E402
from parity_train import build_product, CLARO_AUG  # noqa: E402
from training import augment_mi, loss as loss_mod, trainer as trainer_mod  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ngpu = int(sys.argv[2]) if len(sys.argv) > 2 else 1
second_graphs = (sys.argv[3] != 'eager') if len(sys.argv) > 3 else True
if ngpu > 1:
    class _W:
        def wait(self):
            pass
    torch.distributed.all_reduce = lambda t, async_op=False: (t.mul_(ngpu), _W())[1]
# GRAPH_SKIP=Greg,Dreg: those phases run eagerly in the graph-mode trainer (which phase's graph diverges)
_skip = set(filter(None, os.environ.get('GRAPH_SKIP', '').split(',')))
if _skip:
    _orig = trainer_mod.Trainer._graph_phase

    def _graph_phase(self, phase, ri, rc, gz, gc):
        if phase.name not in _skip:
            return _orig(self, phase, ri, rc, gz, gc)
        phase.opt.zero_grad(set_to_none=True)
        phase.module.requires_grad_(True)
        self._accumulate(phase, ri, rc, gz, gc)
        phase.module.requires_grad_(False)
        return phase.exchange.finish(phase.name, None), False
    trainer_mod.Trainer._graph_phase = _graph_phase
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
                             batch_gpu=cfg['batch'], num_gpus=ngpu, rank=0, device=dev, overlap=ngpu > 1,
                             bucket_mb=0.01 if ngpu > 1 else 32)
    trs.append(tr)
    mods.append((G, D, G_ema))
gen = torch.Generator(device=dev)
gen.manual_seed(5)
for it in range(iters):
    real = torch.rand([cfg['batch'], 1, 32, 32], device=dev, generator=gen) * 2 - 1
    c = torch.nn.functional.one_hot(torch.randint(0, 2, [cfg['batch']], device=dev, generator=gen), 2).float()
    gz = torch.randn([4, cfg['batch'], cfg['z_dim']], device=dev, generator=gen)
    for k, tr in enumerate(trs):
        if it == 1 and k == 1:
            tr.graphs = second_graphs
        torch.manual_seed(123 + it)
        tr.step([real], [c], [[gz[i]] for i in range(4)], [[c] for _ in range(4)])
    torch.cuda.synchronize()
    diffs = []
    for (ga, da, ea), (gb, db, eb) in [(mods[0], mods[1])]:
        for pre, ma, mb in (('G', ga, gb), ('D', da, db), ('G_ema', ea, eb)):
            for (n, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
                diffs.append((float((pa - pb).abs().max()), f'{pre}.{n}'))
    diffs.sort(reverse=True)
    print(f'iter {it}: phases {[p.name for p in trs[1].phases if it % 2 == 0 or not p.name.endswith("reg")]} '
          f'max diff {diffs[0][0]:.3g} at {diffs[0][1]}; next {diffs[1][0]:.3g} {diffs[1][1]}; '
          f'{sum(1 for d, _ in diffs if d > 0)} tensors differ', flush=True)
