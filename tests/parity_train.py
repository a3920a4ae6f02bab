"""Training-iteration parity: product (HIP kernels on cuda:0) vs the CPU oracle and the reference's
golden vectors, on identical weights, inputs and RNG draws (tests/golden/rngtape.py).

Test infrastructure (used by tests/test_train_gpu.py and __graft_entry__.smoke()).
Tolerances: fp32 path (num_fp16_res=0) 1e-4 relative L2 on every gradient / parameter and on
losses (measured worst 3.8e-6); mixed precision (float16 at the top resolutions, the reference's GPU default) 3e-2
on each phase's flat gradient and each network's parameter vector.
"""
import ast
import copy

import numpy as np
import torch

from golden_util import load, rel_err, load_state
from rngtape import Tape


def _T(a, dev):
    return torch.from_numpy(np.array(a, dtype=np.float32)).to(dev)


def build_product(z, dev, fp16):
    from training import networks_stylegan2 as net
    cfg = ast.literal_eval(str(z['cfg']))
    nfp16 = 4 if fp16 else 0
    G = net.Generator(z_dim=cfg['z_dim'], c_dim=cfg['c_dim'], w_dim=cfg['w_dim'], img_resolution=cfg['img_resolution'],
                      img_channels=cfg['img_channels'], channel_base=cfg['channel_base'],
                      channel_max=cfg['channel_max'], num_fp16_res=nfp16, conv_clamp=256,
                      fused_modconv_default='inference_only',
                      mapping_kwargs=dict(num_layers=cfg['map_depth'])).train().requires_grad_(False)
    D = net.Discriminator(c_dim=cfg['c_dim'], img_resolution=cfg['img_resolution'], img_channels=cfg['img_channels'],
                          channel_base=cfg['channel_base'], channel_max=cfg['channel_max'], num_fp16_res=nfp16,
                          conv_clamp=256, epilogue_kwargs=dict(mbstd_group_size=cfg['mbstd'])).train().requires_grad_(False)
    load_state(G, z, 'G0')
    load_state(D, z, 'D0')
    return cfg, G.to(dev), D.to(dev)


CLARO_AUG = dict(xflip=1, xint=1, scale=1, rotate=1, aniso=1, xfrac=1, xint_max=0.05, rotate_max=3 / 360,
                 xfrac_std=0.05, scale_std=0.05, aniso_std=0.05)


def run_product_iteration(z, dev, fp16):
    from training import augment_mi, loss as loss_mod, trainer as trainer_mod
    cfg, G, D = build_product(z, dev, fp16)
    G_ema = copy.deepcopy(G).eval()
    aug = augment_mi.AugmentPipe(run_dir=None, batch_size=cfg['batch'], **CLARO_AUG).train().requires_grad_(False).to(dev)
    aug.p.copy_(torch.as_tensor(0.3))
    loss = loss_mod.StyleGAN2Loss(device=dev, G=G, D=D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9,
                                  pl_weight=2, pl_no_weight_grad=True)
    opt = dict(class_name='torch.optim.Adam', lr=0.0025, betas=[0, 0.99], eps=1e-8)
    tr = trainer_mod.Trainer(G, D, G_ema, loss, opt, opt, batch_size=cfg['batch'], batch_gpu=cfg['batch'],
                             num_gpus=1, rank=0, device=dev)
    grads, stats = {}, []

    def on_grads(name, module):
        for n, p in module.named_parameters():
            if p.grad is not None:
                grads[f'{name}/{n}'] = p.grad.detach().float().cpu().clone()

    tr.on_grads = on_grads
    tr.cur_nimg = 1000
    orig = loss_mod.training_stats.report
    loss_mod.training_stats.report = lambda n, v: (stats.append((n, v.detach().float().cpu().clone())), v)[1]
    tape = Tape.from_npz(z, 'tape')
    try:
        with tape.replay():
            gz = _T(z['gen_z'], dev)
            gc = _T(z['gen_c'], dev)
            tr.step([_T(z['real'], dev)], [_T(z['c'], dev)], [[gz[i]] for i in range(4)], [[gc[i]] for i in range(4)])
        torch.cuda.synchronize()
    finally:
        loss_mod.training_stats.report = orig
    assert tape.pos == len(tape.entries), 'product consumed a different number of random draws'
    return G, D, G_ema, loss, grads, stats


def run_oracle_iteration(z):
    from oracle import sg2_oracle as O
    cfg = ast.literal_eval(str(z['cfg']))
    G = O.Generator(z_dim=cfg['z_dim'], c_dim=cfg['c_dim'], w_dim=cfg['w_dim'], img_resolution=cfg['img_resolution'],
                    img_channels=cfg['img_channels'], channel_base=cfg['channel_base'], channel_max=cfg['channel_max'],
                    num_fp16_res=4, conv_clamp=256, fused_modconv_default='inference_only',
                    mapping_kwargs=dict(num_layers=cfg['map_depth'])).train().requires_grad_(False)
    D = O.Discriminator(c_dim=cfg['c_dim'], img_resolution=cfg['img_resolution'], img_channels=cfg['img_channels'],
                        channel_base=cfg['channel_base'], channel_max=cfg['channel_max'], num_fp16_res=4,
                        conv_clamp=256, epilogue_kwargs=dict(mbstd_group_size=cfg['mbstd'])).train().requires_grad_(False)
    load_state(G, z, 'G0')
    load_state(D, z, 'D0')
    G_ema = copy.deepcopy(G).eval()
    aug = O.AugmentPipe(**CLARO_AUG)
    aug.p.fill_(0.3)
    stats = []
    loss = O.StyleGAN2Loss(None, G, D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9, pl_weight=2,
                           report=lambda n, v: stats.append((n, v.detach().clone())))
    phases = O.make_phases(G, D)
    grads = {}

    def on_grads(name, module):
        for n, p in module.named_parameters():
            if p.grad is not None:
                grads[f'{name}/{n}'] = p.grad.detach().clone()

    tape = Tape.from_npz(z, 'tape')
    T = lambda a: torch.from_numpy(np.array(a, dtype=np.float32))  # noqa: E731
    with tape.replay():
        O.train_iteration(loss, phases, G, G_ema, T(z['real']), T(z['c']), T(z['gen_z']), T(z['gen_c']),
                          batch_idx=0, cur_nimg=1000, batch_size=cfg['batch'], on_grads=on_grads)
    return G, D, G_ema, loss, grads, stats


def run_train_parity(golden='train_claro.npz', fp16=False):
    """Returns the worst relative error; raises AssertionError beyond tolerance."""
    z = load(golden)
    dev = torch.device('cuda', 0)
    tol = 3e-2 if fp16 else 1e-4
    Gp, Dp, Ep, lp, gp, sp = run_product_iteration(z, dev, fp16)
    Go, Do, Eo, lo, go, so = run_oracle_iteration(z)
    worst = 0.0
    # A parameter whose gradient is identically zero may legitimately be absent on one side (the
    # reference's own CUDA and CPU paths differ there); everything else must match one to one.
    for k in set(gp) ^ set(go):
        g = gp.get(k, go.get(k))
        assert float(g.abs().max()) == 0.0, f'gradient {k} present on one side only and non-zero ({float(g.abs().max()):.3g})'
    common = sorted(set(go) & set(gp))
    if not fp16:
        for k in common:
            e = rel_err(gp[k], go[k])
            e2 = rel_err(gp[k], z[f'grad/{k}'])
            worst = max(worst, e, e2)
            assert e <= tol and e2 <= tol, f'grad {k}: rel err vs oracle {e:.3g}, vs reference {e2:.3g} (tol {tol})'
    else:
        # Mixed precision: per phase, the concatenated gradient vector.  Individual tiny gradients (e.g.
        # R1 reaching a bias only through the minibatch-std second derivative) are dominated by fp16
        # rounding, exactly as on the reference's own GPU path, so they are judged inside the whole.
        for ph in ['Gmain', 'Greg', 'Dmain', 'Dreg']:
            ks = [k for k in common if k.startswith(ph + '/')]
            a = torch.cat([gp[k].flatten().double() for k in ks])
            b = torch.cat([go[k].flatten().double() for k in ks])
            e = rel_err(a, b)
            worst = max(worst, e)
            assert e <= tol, f'{ph}: flat gradient rel err {e:.3g} (tol {tol})'
    assert len(sp) == len(so)
    for (n1, v1), (n2, v2) in zip(sp, so):
        assert n1 == n2
        if 'signs' in n1:
            continue
        e = rel_err(v1, v2)
        worst = max(worst, e)
        assert e <= tol, f'stat {n1}: rel err {e:.3g}'
    for (mp, mo) in [(Gp, Go), (Dp, Do), (Ep, Eo)]:
        po = dict(mo.named_parameters())
        if not fp16:
            for n, p in mp.named_parameters():
                e = rel_err(p.detach().float().cpu(), po[n].detach())
                worst = max(worst, e)
                assert e <= tol, f'param {n}: rel err {e:.3g}'
        else:
            # Adam's first step moves every element by ~lr*sign(g); fp16-noisy signs of near-zero
            # gradients flip some of them, so parameters are compared as one vector per network.
            a = torch.cat([p.detach().double().cpu().flatten() for _, p in mp.named_parameters()])
            b = torch.cat([po[n].detach().double().flatten() for n, _ in mp.named_parameters()])
            e = rel_err(a, b)
            worst = max(worst, e)
            assert e <= tol, f'params of {type(mp).__name__}: rel err {e:.3g}'
    e = rel_err(lp.pl_mean.detach().float().cpu(), z['pl_mean'])
    assert e <= tol, f'pl_mean rel err {e:.3g}'
    return worst
