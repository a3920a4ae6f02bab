"""Pin the CPU oracle (oracle/sg2_oracle.py) to golden vectors produced by the REFERENCE itself
(tests/golden/make_golden.py).  CPU only."""
import ast

import numpy as np
import pytest
import torch

from golden_util import load, lit, rel_err, load_state, compare_state
from rngtape import Tape
from oracle import sg2_oracle as O

torch.set_num_threads(4)


def T(a, rg=False):
    return torch.from_numpy(np.array(a, dtype=np.float32)).requires_grad_(rg)


# ------------------------------------------------------------------------------- upfirdn2d
UPF = load('upfirdn2d.npz')


@pytest.mark.parametrize('name', [str(n) for n in UPF['names']])
def test_upfirdn2d(name):
    z = UPF
    kw = lit(z, f'{name}_kw')
    f = z[f'{name}_f']
    f = None if f.size == 0 else torch.from_numpy(f)
    x = T(z[f'{name}_x'], True)
    y = O.upfirdn2d(x, f, **kw)
    assert rel_err(y, z[f'{name}_y']) < 1e-6
    dx, = torch.autograd.grad((y * T(z[f'{name}_dy'])).sum(), [x])
    assert rel_err(dx, z[f'{name}_dx']) < 1e-6


# ------------------------------------------------------------------------------- bias_act
BA = load('bias_act.npz')


@pytest.mark.parametrize('name', [str(n) for n in BA['names']])
def test_bias_act(name):
    z = BA
    act, g, c = name.split('_g')[0], name.split('_g')[1].split('_c')[0], name.split('_c')[1]
    gain = None if g == 'None' else float(g)
    clamp = None if c == 'None' else float(c)
    x, b = T(z['x'], True), T(z['b'], True)
    y = O.bias_act(x, b, act=act, gain=gain, clamp=clamp)
    assert rel_err(y, z[f'{name}_y']) < 1e-6
    gx, gb = torch.autograd.grad((y * T(z['dy'])).sum(), [x, b], create_graph=True)
    assert rel_err(gx, z[f'{name}_dx']) < 1e-6
    assert rel_err(gb, z[f'{name}_db']) < 1e-6
    if f'{name}_ddx' in z.files:
        hx, = torch.autograd.grad((gx * T(z['v'])).sum(), [x])
        assert rel_err(hx, z[f'{name}_ddx']) < 1e-5


# ------------------------------------------------------------------------------- conv
CV = load('conv.npz')


@pytest.mark.parametrize('name', [str(n) for n in CV['names'] if str(n).startswith('modconv')])
def test_modconv(name):
    z = CV
    up = int(name.split('_up')[1][0])
    demod = bool(int(name.split('_d')[1][0]))
    fused = bool(int(name.split('_f')[1][0]))
    x, w, s, nz = (T(z[f'{name}_{k}'], True) for k in ['x', 'w', 's', 'noise'])
    y = O.modulated_conv2d(x, w, s, noise=nz, up=up, padding=1, resample_filter=O.setup_filter([1, 3, 3, 1]),
                           demodulate=demod, flip_weight=(up == 1), fused_modconv=fused)
    assert rel_err(y, z[f'{name}_y']) < 1e-5
    grads = torch.autograd.grad((y * T(z[f'{name}_dy'])).sum(), [x, w, s, nz])
    for k, g in zip(['dx', 'dw', 'ds', 'dnoise'], grads):
        assert rel_err(g, z[f'{name}_{k}']) < 1e-5, k


@pytest.mark.parametrize('name', [str(n) for n in CV['names'] if not str(n).startswith('modconv')])
def test_conv_layer(name):
    z = CV
    kw = lit(z, f'{name}_kw')
    layer = O.Conv2dLayer(**kw)
    with torch.no_grad():
        layer.weight.copy_(T(z[f'{name}_w']))
        if layer.bias is not None:
            layer.bias.copy_(T(z[f'{name}_b']))
    x = T(z[f'{name}_x'], True)
    y = layer(x, gain=float(z[f'{name}_gain']))
    assert rel_err(y, z[f'{name}_y']) < 1e-5
    params = [x, layer.weight] + ([layer.bias] if layer.bias is not None else [])
    grads = torch.autograd.grad((y * T(z[f'{name}_dy'])).sum(), params)
    assert rel_err(grads[0], z[f'{name}_dx']) < 1e-5
    assert rel_err(grads[1], z[f'{name}_dw']) < 1e-5
    if layer.bias is not None:
        assert rel_err(grads[2], z[f'{name}_db']) < 1e-5


# ------------------------------------------------------------------------------- augment
AU = load('augment.npz')


@pytest.mark.parametrize('name', [str(n) for n in AU['names']])
def test_augment(name):
    z = AU
    cfg_name = name.split('_')[0]
    cfg = lit(z, f'{cfg_name}_cfg')
    x = T(z[f'{name}_x'], True)
    pipe = O.AugmentPipe(**cfg)
    if name.endswith('_rand'):
        pipe.p.fill_(float(z[f'{name}_p']))
        tape = Tape.from_npz(z, prefix=f'{name}_tape')
        with tape.replay():
            y = pipe(x, False)
    elif any(k.startswith(f'{name}_tape') for k in z.files):    # the noise branch: pixel noise drawn at any percentile
        tape = Tape.from_npz(z, prefix=f'{name}_tape')
        with tape.replay():
            y = pipe(x, False, debug_percentile=float(name.split('_p')[1]))
        assert tape.pos == len(tape.entries)
    else:
        y = pipe(x, False, debug_percentile=float(name.split('_p')[1]))
    assert rel_err(y, z[f'{name}_y']) < 1e-5
    dx, = torch.autograd.grad((y * T(z[f'{name}_dy'])).sum(), [x])
    assert rel_err(dx, z[f'{name}_dx']) < 1e-5


# ------------------------------------------------------------------------------- network + train iteration
def build_oracle_nets(z):
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
    return cfg, G, D


@pytest.mark.parametrize('tag', ['claro', 'pelvis'])
def test_train_iteration(tag):
    z = load(f'train_{tag}.npz')
    cfg, G, D = build_oracle_nets(z)
    G_ema = O.clone_module(G).eval()
    with torch.no_grad():
        img = G_ema(T(z['z']), T(z['c']), noise_mode='const')
        assert rel_err(img, z['ema_img_const']) < 1e-5
        assert rel_err(D(img, T(z['c'])), z['D_logits_ema']) < 1e-5
        assert rel_err(G_ema.mapping(T(z['z']), T(z['c']), truncation_psi=0.7), z['ws_trunc']) < 1e-6

    from golden_util import load as _  # noqa: F401
    aug = O.AugmentPipe(xflip=1, xint=1, scale=1, rotate=1, aniso=1, xfrac=1, xint_max=0.05, rotate_max=3 / 360,
                        xfrac_std=0.05, scale_std=0.05, aniso_std=0.05)
    aug.p.fill_(0.3)
    stats = []
    loss = O.StyleGAN2Loss(None, G, D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9, pl_weight=2,
                           pl_no_weight_grad=True, report=lambda n, v: stats.append((n, v.detach().clone())))
    phases = O.make_phases(G, D)
    grads = {}

    def on_grads(name, module):
        for n, p in module.named_parameters():
            if p.grad is not None:
                grads[f'{name}/{n}'] = p.grad.detach().clone()

    tape = Tape.from_npz(z, 'tape')
    with tape.replay():
        O.train_iteration(loss, phases, G, G_ema, T(z['real']), T(z['c']), T(z['gen_z']), T(z['gen_c']),
                          batch_idx=0, cur_nimg=1000, batch_size=cfg['batch'], on_grads=on_grads)
    assert tape.pos == len(tape.entries)
    # gradients of every phase
    gkeys = [k for k in z.files if k.startswith('grad/')]
    assert len(gkeys) == len(grads)
    for k in gkeys:
        e = rel_err(grads[k[5:]], z[k])
        assert e < 2e-4, (k, e)
    assert rel_err(loss.pl_mean, z['pl_mean']) < 1e-5
    # reported losses
    for ph in ['Gmain', 'Greg', 'Dmain', 'Dreg']:
        names = [str(s) for s in z[f'stats_names/{ph}']]
        assert names
    flat_ref = [z[f'stats/{ph}/{j}'] for ph in ['Gmain', 'Greg', 'Dmain', 'Dreg']
                for j in range(len(z[f'stats_names/{ph}']))]
    assert len(flat_ref) == len(stats)
    for (n, v), r in zip(stats, flat_ref):
        if 'signs' in n:
            continue
        assert rel_err(v, r) < 1e-4, n
    compare_state(G, z, 'G1', 1e-4)
    compare_state(D, z, 'D1', 1e-4)
    compare_state(G_ema, z, 'Gema1', 1e-4)


# ------------------------------------------------------------------------------- BASELINE configs[0] width
def test_train_iteration_c1_width():
    """The oracle's full iteration at the Claro job's real widths (64^2, cbase 16384 -> 512 channels at
    4^2-32^2, map depth 8, z/w 512, c_dim 2, batch 8) against the reference-generated fixture: per tensor
    against the float64 answer, as close as the reference's own f32 result (config_parity.judge_f32)."""
    from config_parity import load_fixture, run_oracle, judge_f32, judge_stats_f32, judge_pl_mean
    cfg, inp, tape, fix = load_fixture(load('train_c1.npz'))
    got, stats = run_oracle(cfg, inp, tape)
    assert tape.pos == len(tape.entries)
    worst, _ = judge_f32(got, fix)
    judge_stats_f32(stats, fix)
    judge_pl_mean(got, fix)
    print({k: tuple(f'{x:.2g}' for x in v[:4]) for k, v in worst.items() if isinstance(v, tuple)}, worst.get('bound_terms'))
