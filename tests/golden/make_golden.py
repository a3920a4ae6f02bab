"""Generate golden vectors by running the REFERENCE (ltronchin/Gan-track, vendored SG3 code)
on CPU in the build container.  Test infrastructure only; never imported by the product.

Run (from the repo root, build container only -- /root/reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference/src/models/stylegan3:tests/golden:tests:. \
        python tests/golden/make_golden.py [ops] [nets] [c1] [c2] [c4] [c5]

Harness shims; the reference tree itself is not modified:
  * ``openpyxl`` is stubbed (imported by genlib/utils/util_general.py:8, unused on this path);
  * ``torch._C._jit_get_operation('aten::grid_sampler_2d_backward')`` returns a tuple on
    torch>=1.13; SG3/torch_utils/ops/grid_sample_gradfix.py:60 expects the op itself;
  * ``conv2d_gradfix.enabled = grid_sample_gradfix.enabled = True`` as the training loop does
    (SG3/training/training_loop_mi_multimodal.py:171-172).
Never called: training_loop()/main() (IFTTT HTTP notify, util_general.py:76-79) or any metric.

Outputs: tests/golden/*.npz (small, committed).
"""
import copy
import zlib
import os
import re
import sys
import types

import numpy as np

sys.modules['openpyxl'] = types.ModuleType('openpyxl')
import torch  # noqa: E402

_orig_jit_get = torch._C._jit_get_operation


def _jit_get(name):
    r = _orig_jit_get(name)
    if name == 'aten::grid_sampler_2d_backward' and isinstance(r, tuple):
        return r[0]
    return r


torch._C._jit_get_operation = _jit_get

from torch_utils.ops import upfirdn2d, bias_act, conv2d_gradfix, grid_sample_gradfix  # noqa: E402
from torch_utils import training_stats  # noqa: E402
from training import networks_stylegan2 as net  # noqa: E402
from training import augment_mi  # noqa: E402
from training import loss as loss_mod  # noqa: E402
from rngtape import Tape  # noqa: E402
from golden_init import init_state, summarize, pack  # noqa: E402

conv2d_gradfix.enabled = True
grid_sample_gradfix.enabled = True
torch.set_num_threads(min(8, os.cpu_count()))

OUT = os.path.dirname(os.path.abspath(__file__))


def rs(seed):
    return np.random.RandomState(seed)


def T(a, rg=False):
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
    return t.requires_grad_(rg)


def npy(t):
    return t.detach().cpu().numpy().astype(np.float32)


# ---------------------------------------------------------------------------- upfirdn2d
def gen_upfirdn2d():
    d = {}
    f4 = upfirdn2d.setup_filter([1, 3, 3, 1])
    sym6 = upfirdn2d.setup_filter(augment_mi.wavelets['sym6'])
    cases = [
        # name, x shape, f, kwargs
        ('up2', (2, 3, 7, 9), f4, dict(up=2, padding=[2, 1, 2, 1], gain=4)),                 # upsample2d (networks_stylegan2.py:451)
        ('down2', (2, 3, 10, 12), f4, dict(down=2, padding=[1, 1, 1, 1])),                   # downsample2d / D skip
        ('pad2', (2, 3, 8, 8), f4, dict(padding=[2, 2, 2, 2])),                              # D conv1 pre-filter
        ('convT', (2, 3, 9, 9), f4, dict(padding=[1, 1, 1, 1], gain=4)),                     # G conv0 post transposed conv
        ('sep_up2', (2, 2, 11, 10), sym6, dict(up=2, padding=[6, 5, 6, 5], gain=4)),        # ADA upsample2d(Hz_geom)
        ('sep_down2', (2, 2, 30, 28), sym6, dict(down=2, padding=[-1, -1, -1, -1], flip_filter=True)),  # ADA downsample2d
        ('generic', (1, 2, 6, 5), upfirdn2d.setup_filter([[1, 2, 0], [3, 1, 1], [0, 2, 5]], normalize=False),
         dict(up=[3, 2], down=[2, 1], padding=[2, -1, 1, 3], flip_filter=True, gain=2.0)),
        ('ident', (2, 3, 5, 6), None, dict(padding=[1, 0, 0, 2])),
    ]
    for i, (name, shape, f, kw) in enumerate(cases):
        r = rs(100 + i)
        x = T(r.standard_normal(shape), rg=True)
        y = upfirdn2d.upfirdn2d(x, f, impl='ref', **kw)
        dy = r.standard_normal(tuple(y.shape)).astype(np.float32)
        dx, = torch.autograd.grad((y * T(dy)).sum(), [x])
        d[f'{name}_x'] = npy(x)
        d[f'{name}_f'] = np.zeros([0], np.float32) if f is None else npy(f)
        d[f'{name}_y'] = npy(y)
        d[f'{name}_dy'] = dy
        d[f'{name}_dx'] = npy(dx)
        d[f'{name}_kw'] = np.array(repr(kw))
    d['names'] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(OUT, 'upfirdn2d.npz'), **d)


# ---------------------------------------------------------------------------- bias_act
def gen_bias_act():
    d = {}
    names = []
    r = rs(7)
    x0 = r.standard_normal((3, 5, 4, 6)).astype(np.float32) * 2
    b0 = r.standard_normal((5,)).astype(np.float32)
    dy0 = r.standard_normal((3, 5, 4, 6)).astype(np.float32)
    v0 = r.standard_normal((3, 5, 4, 6)).astype(np.float32)
    d['x'], d['b'], d['dy'], d['v'] = x0, b0, dy0, v0
    for act in bias_act.activation_funcs:
        for gain, clamp in [(None, None), (0.7, None), (None, 0.9)]:
            name = f'{act}_g{gain}_c{clamp}'
            names.append(name)
            x = T(x0, rg=True)
            b = T(b0, rg=True)
            y = bias_act.bias_act(x, b, act=act, gain=gain, clamp=clamp, impl='ref')
            gx, gb = torch.autograd.grad((y * T(dy0)).sum(), [x, b], create_graph=True)
            d[f'{name}_y'] = npy(y)
            d[f'{name}_dx'] = npy(gx)
            d[f'{name}_db'] = npy(gb)
            spec = bias_act.activation_funcs[act]
            if spec.has_2nd_grad:
                # d/dx <dx, v>  (second-order through the activation; SG3 bias_act.py:175-203)
                hx, = torch.autograd.grad((gx * T(v0)).sum(), [x])
                d[f'{name}_ddx'] = npy(hx)
    d['names'] = np.array(names)
    np.savez_compressed(os.path.join(OUT, 'bias_act.npz'), **d)


# ---------------------------------------------------------------------------- modulated conv + conv layers
def gen_conv():
    d = {}
    f4 = upfirdn2d.setup_filter([1, 3, 3, 1])
    names = []
    for up in [1, 2]:
        for demod in [True, False]:
            for fused in [False, True]:
                name = f'modconv_up{up}_d{int(demod)}_f{int(fused)}'
                names.append(name)
                r = rs(zlib.crc32(name.encode()) % 1000)
                res_in = 6 if up == 1 else 4
                res_out = res_in * up
                x = T(r.standard_normal((2, 4, res_in, res_in)), rg=True)
                w = T(r.standard_normal((5, 4, 3, 3)), rg=True)
                s = T(r.standard_normal((2, 4)) + 1.0, rg=True)
                noise = T(r.standard_normal((2, 1, res_out, res_out)) * 0.3, rg=True)
                y = net.modulated_conv2d(x=x, weight=w, styles=s, noise=noise, up=up, padding=1,
                                         resample_filter=f4, demodulate=demod, flip_weight=(up == 1),
                                         fused_modconv=fused)
                dy = r.standard_normal(tuple(y.shape)).astype(np.float32)
                gx, gw, gs, gn = torch.autograd.grad((y * T(dy)).sum(), [x, w, s, noise])
                for k, v in dict(x=x, w=w, s=s, noise=noise, y=y, dx=gx, dw=gw, ds=gs, dnoise=gn).items():
                    d[f'{name}_{k}'] = npy(v)
                d[f'{name}_dy'] = dy
    # Discriminator-style conv layers (SG3 networks_stylegan2.py:133-181 -> conv2d_resample.py:46-141)
    layer_cfgs = [
        ('conv3', dict(in_channels=4, out_channels=6, kernel_size=3, activation='lrelu', conv_clamp=256), 8),
        ('conv3_down', dict(in_channels=4, out_channels=6, kernel_size=3, activation='lrelu', down=2, conv_clamp=256), 8),
        ('skip_down', dict(in_channels=4, out_channels=6, kernel_size=1, bias=False, down=2), 8),
        ('fromrgb', dict(in_channels=1, out_channels=6, kernel_size=1, activation='lrelu', conv_clamp=256), 8),
        ('skip_up', dict(in_channels=4, out_channels=6, kernel_size=1, bias=False, up=2), 4),
        ('conv3_up', dict(in_channels=4, out_channels=6, kernel_size=3, activation='lrelu', up=2), 4),
    ]
    for name, kw, res in layer_cfgs:
        names.append(name)
        torch.manual_seed(11)
        layer = net.Conv2dLayer(**kw)
        with torch.no_grad():
            if layer.bias is not None:
                layer.bias.copy_(torch.randn(layer.bias.shape) * 0.2)
        r = rs(zlib.crc32(name.encode()) % 1000)
        x = T(r.standard_normal((2, kw['in_channels'], res, res)), rg=True)
        gain = 0.7071067811865476 if name.startswith('skip') else 1
        y = layer(x, gain=gain)
        dy = r.standard_normal(tuple(y.shape)).astype(np.float32)
        params = [layer.weight] + ([layer.bias] if layer.bias is not None else [])
        grads = torch.autograd.grad((y * T(dy)).sum(), [x] + params)
        d[f'{name}_x'] = npy(x)
        d[f'{name}_w'] = npy(layer.weight)
        d[f'{name}_b'] = npy(layer.bias) if layer.bias is not None else np.zeros([0], np.float32)
        d[f'{name}_y'] = npy(y)
        d[f'{name}_dy'] = dy
        d[f'{name}_dx'] = npy(grads[0])
        d[f'{name}_dw'] = npy(grads[1])
        d[f'{name}_db'] = npy(grads[2]) if len(grads) > 2 else np.zeros([0], np.float32)
        d[f'{name}_kw'] = np.array(repr(kw))
        d[f'{name}_gain'] = np.array(gain, np.float32)
    d['names'] = np.array(names)
    np.savez_compressed(os.path.join(OUT, 'conv.npz'), **d)


# ---------------------------------------------------------------------------- augment pipe
CLARO_AUG = dict(xflip=1, xint=1, scale=1, rotate=1, aniso=1, xfrac=1,
                 xint_max=0.05, rotate_max=3 / 360, xfrac_std=0.05, scale_std=0.05, aniso_std=0.05)
FULL_AUG = dict(xflip=1, rotate90=1, xint=1, scale=1, rotate=1, aniso=1, xfrac=1,
                brightness=1, contrast=1, lumaflip=1, hue=1, saturation=1, imgfilter=1, cutout=1)


def gen_augment():
    d = {}
    names = []
    for cfg_name, cfg, shape in [('claro', CLARO_AUG, (2, 1, 32, 32)), ('full3', FULL_AUG, (2, 3, 24, 24)),
                                 ('full1', FULL_AUG, (2, 1, 28, 28)),
                                 # + the additive-noise branch (augment_mi.py:427-433), which FULL_AUG leaves out
                                 ('noise3', dict(FULL_AUG, noise=1), (2, 3, 24, 24))]:
        pipe = augment_mi.AugmentPipe(run_dir=None, batch_size=shape[0], **cfg)
        d[f'{cfg_name}_cfg'] = np.array(repr(cfg))
        for pct in [0.1, 0.5, 0.9]:
            name = f'{cfg_name}_p{pct}'
            names.append(name)
            r = rs(int(pct * 100) + len(cfg))
            x = T(r.uniform(-1, 1, shape), rg=True)
            if cfg.get('noise', 0):
                # the noise branch draws its pixel noise even at a debug percentile (augment_mi.py:431): record it
                tape = Tape(seed=11)
                with tape.record():
                    y = pipe(x, False, debug_percentile=pct)
                d.update(tape.to_npz_dict(prefix=f'{name}_tape'))
            else:
                y = pipe(x, False, debug_percentile=pct)
            dy = r.standard_normal(tuple(y.shape)).astype(np.float32)
            gx, = torch.autograd.grad((y * T(dy)).sum(), [x])
            d[f'{name}_x'] = npy(x)
            d[f'{name}_y'] = npy(y)
            d[f'{name}_dy'] = dy
            d[f'{name}_dx'] = npy(gx)
        # random (non-debug) path, RNG recorded on a tape
        name = f'{cfg_name}_rand'
        names.append(name)
        pipe.p.fill_(0.6)
        r = rs(77)
        x = T(r.uniform(-1, 1, shape), rg=True)
        tape = Tape(seed=5)
        with tape.record():
            y = pipe(x, False)
        dy = r.standard_normal(tuple(y.shape)).astype(np.float32)
        gx, = torch.autograd.grad((y * T(dy)).sum(), [x])
        d[f'{name}_x'] = npy(x)
        d[f'{name}_y'] = npy(y)
        d[f'{name}_dy'] = dy
        d[f'{name}_dx'] = npy(gx)
        d[f'{name}_p'] = np.array(0.6, np.float32)
        d.update(tape.to_npz_dict(prefix=f'{name}_tape'))
    d['names'] = np.array(names)
    np.savez_compressed(os.path.join(OUT, 'augment.npz'), **d)


# ---------------------------------------------------------------------------- networks + one training iteration
NET_CFG = dict(z_dim=32, w_dim=32, img_resolution=32, channel_base=128, channel_max=16, map_depth=8, mbstd=4, batch=4)


def _state(module):
    return {k: npy(v) for k, v in list(module.named_parameters()) + list(module.named_buffers())}


def gen_network(c_dim, img_channels, tag):
    cfg = NET_CFG
    d = {}
    torch.manual_seed(0)
    G = net.Generator(z_dim=cfg['z_dim'], c_dim=c_dim, w_dim=cfg['w_dim'], img_resolution=cfg['img_resolution'],
                      img_channels=img_channels, channel_base=cfg['channel_base'], channel_max=cfg['channel_max'],
                      num_fp16_res=4, conv_clamp=256, fused_modconv_default='inference_only',
                      mapping_kwargs=dict(num_layers=cfg['map_depth'])).train().requires_grad_(False)
    D = net.Discriminator(c_dim=c_dim, img_resolution=cfg['img_resolution'], img_channels=img_channels,
                          channel_base=cfg['channel_base'], channel_max=cfg['channel_max'], num_fp16_res=4,
                          conv_clamp=256, block_kwargs=dict(freeze_layers=0), mapping_kwargs=dict(),
                          epilogue_kwargs=dict(mbstd_group_size=cfg['mbstd'])).train().requires_grad_(False)
    # Non-trivial noise strengths and biases so every gradient path carries signal.
    with torch.no_grad():
        for n_, p in G.named_parameters():
            if n_.endswith('noise_strength'):
                p.fill_(0.1)
            elif n_.endswith('.bias') and 'affine' not in n_ and 'mapping' not in n_:
                p.copy_(torch.randn(p.shape) * 0.1)
        for n_, p in D.named_parameters():
            if n_.endswith('.bias'):
                p.copy_(torch.randn(p.shape) * 0.1)
    G_ema = copy.deepcopy(G).eval()
    for k, v in _state(G).items():
        d[f'G0/{k}'] = v
    for k, v in _state(D).items():
        d[f'D0/{k}'] = v

    B = cfg['batch']
    r = rs(3)
    z = r.standard_normal((B, cfg['z_dim'])).astype(np.float32)
    c = np.eye(max(c_dim, 1), dtype=np.float32)[r.randint(max(c_dim, 1), size=B)][:, :c_dim]
    real = r.uniform(-1, 1, (B, img_channels, cfg['img_resolution'], cfg['img_resolution'])).astype(np.float32)
    d['z'], d['c'], d['real'] = z, c, real

    # Inference forward (G_ema, noise_mode='const', fused modconv) + D logits.
    with torch.no_grad():
        img = G_ema(T(z), T(c), noise_mode='const')
        logits = D(img, T(c))
        ws = G_ema.mapping(T(z), T(c), truncation_psi=0.7)
    d['ema_img_const'] = npy(img)
    d['D_logits_ema'] = npy(logits)
    d['ws_trunc'] = npy(ws)

    # One full training iteration mirroring SG3 training_loop_mi_multimodal.py:326-366
    aug = augment_mi.AugmentPipe(run_dir=None, batch_size=B, **CLARO_AUG).train().requires_grad_(False)
    aug.p.copy_(torch.as_tensor(0.3))
    stats = []
    orig_report = training_stats.report

    def rep(name, value):
        stats.append((name, npy(torch.as_tensor(value))))
        return value

    loss_mod.training_stats.report = rep
    loss = loss_mod.StyleGAN2Loss(device=torch.device('cpu'), G=G, D=D, augment_pipe=aug, r1_gamma=0.4096,
                                  style_mixing_prob=0.9, pl_weight=2, pl_no_weight_grad=True)
    phases = []
    for name, module, reg_interval, lr in [('G', G, 4, 0.0025), ('D', D, 16, 0.0025)]:
        mb_ratio = reg_interval / (reg_interval + 1)
        opt = torch.optim.Adam(module.parameters(), lr=lr * mb_ratio, betas=[b ** mb_ratio for b in [0, 0.99]], eps=1e-8)
        phases += [dict(name=name + 'main', module=module, opt=opt, interval=1)]
        phases += [dict(name=name + 'reg', module=module, opt=opt, interval=reg_interval)]
    gen_z = r.standard_normal((len(phases), B, cfg['z_dim'])).astype(np.float32)
    gen_c = np.eye(max(c_dim, 1), dtype=np.float32)[r.randint(max(c_dim, 1), size=(len(phases), B))][..., :c_dim]
    d['gen_z'], d['gen_c'] = gen_z, gen_c
    cur_nimg = 1000
    tape = Tape(seed=9)
    with tape.record():
        for pi, ph in enumerate(phases):
            ph['opt'].zero_grad(set_to_none=True)
            ph['module'].requires_grad_(True)
            n0 = len(stats)
            loss.accumulate_gradients(phase=ph['name'], real_img=T(real), real_c=T(c), gen_z=T(gen_z[pi]),
                                      gen_c=T(gen_c[pi]), gain=ph['interval'], cur_nimg=cur_nimg)
            ph['module'].requires_grad_(False)
            params = [p for p in ph['module'].parameters() if p.grad is not None]
            flat = torch.cat([p.grad.flatten() for p in params])
            torch.nan_to_num(flat, nan=0, posinf=1e5, neginf=-1e5, out=flat)
            for p, g in zip(params, flat.split([p.numel() for p in params])):
                p.grad = g.reshape(p.shape)
            named = dict(ph['module'].named_parameters())
            inv = {id(v): k for k, v in named.items()}
            for p in params:
                d[f'grad/{ph["name"]}/{inv[id(p)]}'] = npy(p.grad)
            ph['opt'].step()
            d[f'stats_names/{ph["name"]}'] = np.array([s[0] for s in stats[n0:]])
            for j, s in enumerate(stats[n0:]):
                d[f'stats/{ph["name"]}/{j}'] = s[1]
            if ph['name'] == 'Greg':
                d['pl_mean'] = npy(loss.pl_mean)
    loss_mod.training_stats.report = orig_report
    ema_nimg = min(10 * 1000, cur_nimg * 0.05)
    ema_beta = 0.5 ** (B / max(ema_nimg, 1e-8))
    with torch.no_grad():
        for p_ema, p in zip(G_ema.parameters(), G.parameters()):
            p_ema.copy_(p.lerp(p_ema, ema_beta))
        for b_ema, b in zip(G_ema.buffers(), G.buffers()):
            b_ema.copy_(b)
    d['ema_beta'] = np.array(ema_beta, np.float64)
    for k, v in _state(G).items():
        d[f'G1/{k}'] = v
    for k, v in _state(D).items():
        d[f'D1/{k}'] = v
    for k, v in _state(G_ema).items():
        d[f'Gema1/{k}'] = v
    d.update(tape.to_npz_dict('tape'))
    d['cfg'] = np.array(repr(dict(NET_CFG, c_dim=c_dim, img_channels=img_channels)))
    np.savez_compressed(os.path.join(OUT, f'train_{tag}.npz'), **d)


# ---------------------------------------------------------------------------- configuration-width iterations
# One full iteration at each BASELINE.json configuration's real width, through the REFERENCE (fp32 CPU,
# as its CPU path runs) and through the oracle in float64 (the rounding-free answer both fp32 results
# are judged against).  Full-width networks are too large to commit, so the state is derived from the
# parameter names (golden_init.init_state), the inputs from a seed (config_parity.make_inputs), the RNG
# tape is stored as its seed, and the results as norms + sampled entries (golden_init.summarize).
CONFIGS = {
    # configs[0]: claro_stylegan2-ada.yaml / the Claro job at 64^2 (cbase 16384, map 8, c_dim 2, batch 8)
    'c1': dict(z_dim=512, w_dim=512, img_resolution=64, channel_base=16384, channel_max=512, map_depth=8, mbstd=4,
               batch=8, c_dim=2, img_channels=1),
    # configs[1..2]: the 256^2 1-ch Claro network (batch 4 of the per-GPU 32: CPU time)
    'c2': dict(z_dim=512, w_dim=512, img_resolution=256, channel_base=16384, channel_max=512, map_depth=8, mbstd=4,
               batch=4, c_dim=2, img_channels=1),
    # configs[3]: 512^2 3-ch, cbase 32768 (batch 2 of 16)
    'c4': dict(z_dim=512, w_dim=512, img_resolution=512, channel_base=32768, channel_max=512, map_depth=8, mbstd=4,
               batch=2, c_dim=0, img_channels=3),
    # configs[4]: 1024^2 3-ch, cbase 32768 (batch 2 of 8)
    'c5': dict(z_dim=512, w_dim=512, img_resolution=1024, channel_base=32768, channel_max=512, map_depth=8, mbstd=4,
               batch=2, c_dim=0, img_channels=3),
}


def gen_config_iteration(tag, cfg, input_seed=31, tape_seed=13, aug_p=0.3, isolated=False):
    """isolated: the phase-isolated fixture train_<tag>_iso.npz -- every phase from the initial state (parameters
    and buffers restored, no optimiser step), see oracle.sg2_oracle.train_iteration."""
    import config_parity as cp
    d = {}
    torch.manual_seed(0)
    c_dim, img_channels = cfg['c_dim'], cfg['img_channels']
    G = net.Generator(z_dim=cfg['z_dim'], c_dim=c_dim, w_dim=cfg['w_dim'], img_resolution=cfg['img_resolution'],
                      img_channels=img_channels, channel_base=cfg['channel_base'], channel_max=cfg['channel_max'],
                      num_fp16_res=4, conv_clamp=256, fused_modconv_default='inference_only',
                      mapping_kwargs=dict(num_layers=cfg['map_depth'])).train().requires_grad_(False)
    D = net.Discriminator(c_dim=c_dim, img_resolution=cfg['img_resolution'], img_channels=img_channels,
                          channel_base=cfg['channel_base'], channel_max=cfg['channel_max'], num_fp16_res=4,
                          conv_clamp=256, epilogue_kwargs=dict(mbstd_group_size=cfg['mbstd'])).train().requires_grad_(False)
    init_state(G, seed=1)
    init_state(D, seed=2)
    G_ema = copy.deepcopy(G).eval()
    B = cfg['batch']
    inp = cp.make_inputs(cfg, input_seed)
    if cfg['img_resolution'] <= 64:
        with torch.no_grad():
            img = G_ema(T(inp['z']), T(inp['c']), noise_mode='const')
            d['ema_img_const'] = npy(img)
            d['D_logits_ema'] = npy(D(img, T(inp['c'])))
    aug = augment_mi.AugmentPipe(run_dir=None, batch_size=B, **CLARO_AUG).train().requires_grad_(False)
    aug.p.copy_(torch.as_tensor(aug_p))
    stats = []

    def rep(name, value):
        stats.append((name, npy(torch.as_tensor(value))))
        return value

    orig_report = training_stats.report
    loss_mod.training_stats.report = rep
    loss = loss_mod.StyleGAN2Loss(device=torch.device('cpu'), G=G, D=D, augment_pipe=aug, r1_gamma=0.4096,
                                  style_mixing_prob=0.9, pl_weight=2, pl_no_weight_grad=True)
    phases = []
    for name, module, reg_interval in [('G', G, 4), ('D', D, 16)]:
        mb_ratio = reg_interval / (reg_interval + 1)
        opt = torch.optim.Adam(module.parameters(), lr=0.0025 * mb_ratio, betas=[b ** mb_ratio for b in [0, 0.99]],
                               eps=1e-8)
        phases += [dict(name=name + 'main', module=module, opt=opt, interval=1),
                   dict(name=name + 'reg', module=module, opt=opt, interval=reg_interval)]
    gen_z, gen_c = inp['gen_z'], inp['gen_c']
    cur_nimg = 1000
    tape = Tape(seed=tape_seed)
    start = [{k: v.detach().clone() for k, v in m.state_dict().items()} for m in (G, D)]
    with tape.record():
        for pi, ph in enumerate(phases):
            if isolated:
                with torch.no_grad():
                    for m, sd in zip((G, D), start):
                        for k, v in m.state_dict().items():
                            v.copy_(sd[k])
            ph['opt'].zero_grad(set_to_none=True)
            ph['module'].requires_grad_(True)
            n0 = len(stats)
            loss.accumulate_gradients(phase=ph['name'], real_img=T(inp['real']), real_c=T(inp['c']),
                                      gen_z=T(gen_z[pi]), gen_c=T(gen_c[pi]), gain=ph['interval'], cur_nimg=cur_nimg)
            ph['module'].requires_grad_(False)
            named = [(n_, p) for n_, p in ph['module'].named_parameters() if p.grad is not None]
            flat = torch.cat([p.grad.flatten() for _, p in named])
            torch.nan_to_num(flat, nan=0, posinf=1e5, neginf=-1e5, out=flat)
            for (_, p), g in zip(named, flat.split([p.numel() for _, p in named])):
                p.grad = g.reshape(p.shape)
            d.update(summarize({n_: p.grad for n_, p in named}, f'grad/{ph["name"]}'))
            if not isolated:
                ph['opt'].step()
            d[f'stats_names/{ph["name"]}'] = np.array([s_[0] for s_ in stats[n0:]])
            for j, s_ in enumerate(stats[n0:]):
                d[f'stats/{ph["name"]}/{j}'] = s_[1]
            if ph['name'] == 'Greg':
                d['pl_mean'] = npy(loss.pl_mean)
    loss_mod.training_stats.report = orig_report
    if not isolated:
        ema_beta = 0.5 ** (B / max(min(10 * 1000, cur_nimg * 0.05), 1e-8))
        with torch.no_grad():
            for p_ema, p in zip(G_ema.parameters(), G.parameters()):
                p_ema.copy_(p.lerp(p_ema, ema_beta))
        d.update(summarize(dict(G.named_parameters()), 'G1'))
        d.update(summarize(dict(D.named_parameters()), 'D1'))
        d.update(summarize(dict(G_ema.named_parameters()), 'Gema1'))
    d.update(tape.to_compact_npz_dict('tape'))
    # the float64 oracle on the same state, inputs and draws
    replay = Tape.from_npz(tape.to_compact_npz_dict('t'), 't')
    f64, f64_stats = cp.run_oracle_f64(cfg, inp, replay, aug_p, isolated=isolated)
    assert replay.pos == len(replay.entries)
    for k, v in f64.items():
        d[f'f64/{k}'] = v
    for j, (n_, v) in enumerate(f64_stats):
        d[f'f64/stats/{j}'] = np.asarray(v, np.float64)
    d['cfg'] = np.array(repr(dict(cfg, aug_p=aug_p, init_seeds=(1, 2), input_seed=input_seed, isolated=isolated)))
    np.savez_compressed(os.path.join(OUT, f'train_{tag}{"_iso" if isolated else ""}.npz'), **pack(d))
    print(tag, 'written', flush=True)


# The same widths with the ADA pipe at p = 0: every augmentation's probability is zero, so no discrete choice
# (integer translation, flips, the reflect-pad margins) can come out differently in f32 and in float64 -- the
# geometric branch still runs (pad, sym6 up-sampling, identity warp, down-sampling), so R1's double backward
# still goes through grid_sample.  These fixtures separate rounding from the p = 0.3 fixtures' discrete flips.
P0_CONFIGS = {f'{k}p0': k for k in ('c2', 'c4', 'c5')}


def gen_conditioning(tag, cache_dir=None, perturb=2.0 ** -24):
    """Add 'f64p/...' to train_<tag>.npz: the float64 oracle on the fixture's state, inputs and draws with
    every parameter, real image and latent nudged by a factor (1 +- 2^-24) -- half an f32 ulp, a fixed random
    sign per entry (config_parity.run_oracle).  How far that moves each result from the float64 answer is the
    conditioning any f32 evaluation inherits: measured at C2 / ADA p = 0 it moves the R1 (Dreg) flat gradient
    by 1.6 % and its bias gradients by 5-17 %, the size of the reference's own f32 error there
    (profiles/r03_conditioning.txt).  The GPU tests bound each tensor by it (config_parity.judge_cond).
    Oracle only; slow (C2 ~17 min on 8 cores).  cache_dir: reuse a saved f64p_<tag>.npz."""
    import config_parity as cp
    from golden_init import unpack
    path = os.path.join(OUT, f'train_{tag}.npz')
    with np.load(path, allow_pickle=False) as f:
        z = unpack(f)
    z = {k: v for k, v in z.items() if not k.startswith('f64p/')}
    with np.load(path, allow_pickle=False) as f:
        cfg, inp, tape, _ = cp.load_fixture(f)
    cached = os.path.join(cache_dir, f'f64p_{tag}.npz') if cache_dir else None
    if cached and os.path.exists(cached):
        with np.load(cached, allow_pickle=False) as f:
            out = unpack(f)
    else:
        out, _ = cp.run_oracle_f64(cfg, inp, tape, cfg.get('aug_p', 0.3), perturb=perturb,
                                   isolated=cfg.get('isolated', False))
    z.update({f'f64p/{k}': v for k, v in out.items()})
    z['f64p_perturb'] = np.array(perturb, np.float64)
    np.savez_compressed(path, **pack(z))
    print(tag, 'conditioning written', flush=True)

def gen_emulated16_nudged(tag, dt, seed, cache_dir):
    """One more sample of the emulated reference 16-bit evaluation: the same emulation (oracle EMU16) at the
    fixture's state nudged by (1 +- 2^-24) (seeded signs; a state equal within f32 rounding), saved to
    <cache_dir>/q16n_<tag>_<dt>_<seed>.npz; emu16merge folds the samples in as '<q16|qbf>n<seed>/...'.  The spread of
    these samples is the reference's own 16-bit spread on each error measure (tests/test_config_gpu.py)."""
    import config_parity as cp
    path = os.path.join(OUT, f'train_{tag}.npz')
    with np.load(path, allow_pickle=False) as f:
        cfg, inp, tape, _ = cp.load_fixture(f)
    out, _ = cp.run_oracle_f64(cfg, inp, tape, cfg.get('aug_p', 0.3), perturb=2.0 ** -24, perturb_seed=int(seed),
                               isolated=cfg.get('isolated', False),
                               emu16={'fp16': torch.float16, 'bf16': torch.bfloat16}[dt])
    os.makedirs(cache_dir, exist_ok=True)
    np.savez_compressed(os.path.join(cache_dir, f'q16n_{tag}_{dt}_{seed}.npz'), **pack(out))
    print(tag, dt, seed, 'nudged 16-bit emulation sample written', flush=True)


def merge_emulated16_nudged(tag, cache_dir):
    from golden_init import unpack
    import glob
    path = os.path.join(OUT, f'train_{tag}.npz')
    with np.load(path, allow_pickle=False) as f:
        z = unpack(f)
    z = {k: v for k, v in z.items() if not (k.startswith(('q16n', 'qbfn')))}
    n = 0
    for fn in sorted(glob.glob(os.path.join(cache_dir, f'q16n_{tag}_*.npz'))):
        dt, seed = fn[:-4].rsplit('_', 2)[1:]
        pre = {'fp16': 'q16', 'bf16': 'qbf'}[dt] + 'n' + seed
        with np.load(fn, allow_pickle=False) as f:
            z.update({f'{pre}/{k}': v for k, v in unpack(f).items()})
        n += 1
    tmp = path + '.tmp.npz'
    np.savez_compressed(tmp, **pack(z))
    os.replace(tmp, path)              # (atomic: a concurrent reader sees the old or the new file)
    print(tag, n, 'nudged 16-bit emulation samples merged', flush=True)


def gen_emulated16_perturbed(tag, dts, seed, k, cache_dir):
    """Same-state samples for the 16-bit comparison: the fixture's state nudged by (1 +- 2^-k) (seeded signs;
    k = 12 moves each entry by 1/16 of a bf16 ulp, so every sample redraws the 16-bit rounding pattern, which the
    half-f32-ulp nudges of emu16n do not), the float64 answer at that state and the emulated reference's 16-bit
    evaluation of it in each type of `dts`, saved to <cache_dir>/p<k>_<tag>_<f64|fp16|bf16>_<seed>.npz;
    emu16pmerge folds them in as 'f64p<k>s<seed>/', 'q16p<k>s<seed>/', 'qbfp<k>s<seed>/'.  The product runs at the
    same states (config_parity.run_product perturb: the same signs in the same order, the state rounded to f32)."""
    import config_parity as cp
    path = os.path.join(OUT, f'train_{tag}.npz')
    os.makedirs(cache_dir, exist_ok=True)
    for dt in ['f64'] + list(dts):
        fn = os.path.join(cache_dir, f'p{k}_{tag}_{dt}_{seed}.npz')
        if os.path.exists(fn):
            continue
        with np.load(path, allow_pickle=False) as f:
            cfg, inp, tape, _ = cp.load_fixture(f)
        out, _ = cp.run_oracle_f64(cfg, inp, tape, cfg.get('aug_p', 0.3), perturb=2.0 ** -k, perturb_seed=int(seed),
                                   isolated=cfg.get('isolated', False),
                                   emu16=None if dt == 'f64' else {'fp16': torch.float16, 'bf16': torch.bfloat16}[dt])
        tmp = fn + '.tmp.npz'
        np.savez_compressed(tmp, **pack(out))
        os.replace(tmp, fn)
        print(tag, dt, k, seed, 'perturbed sample written', flush=True)


def merge_emulated16_perturbed(tag, cache_dir):
    from golden_init import unpack
    import glob
    path = os.path.join(OUT, f'train_{tag}.npz')
    with np.load(path, allow_pickle=False) as f:
        z = unpack(f)
    z = {kk: v for kk, v in z.items() if not re.match(r'(f64|q16|qbf)p\d+s\d+/', kk)}
    n = 0
    for fn in sorted(glob.glob(os.path.join(cache_dir, f'p*_{tag}_*.npz'))):
        m = re.match(r'p(\d+)_' + re.escape(tag) + r'_(f64|fp16|bf16)_(\d+)\.npz$', os.path.basename(fn))
        if not m:
            continue
        pre = {'f64': 'f64', 'fp16': 'q16', 'bf16': 'qbf'}[m.group(2)] + f'p{m.group(1)}s{m.group(3)}'
        with np.load(fn, allow_pickle=False) as f:
            z.update({f'{pre}/{kk}': v for kk, v in unpack(f).items()})
        n += 1
    tmp = path + '.tmp.npz'
    np.savez_compressed(tmp, **pack(z))
    os.replace(tmp, path)
    print(tag, n, 'perturbed samples merged', flush=True)


def gen_emulated16(tag, dt):
    """Add 'q16/...' (dt fp16) or 'qbf/...' (bf16) to train_<tag>.npz: the oracle's emulation of the reference's
    16-bit GPU evaluation of the fixture (oracle.sg2_oracle.EMU16: the num_fp16_res = 4 blocks round every tensor
    and gradient where the reference's fp16 blocks do), float64 otherwise.  Its distance from the float64 answer
    is the reference's own 16-bit error, the yardstick of the product's 16-bit tests."""
    import config_parity as cp
    from golden_init import unpack
    path = os.path.join(OUT, f'train_{tag}.npz')
    with np.load(path, allow_pickle=False) as f:
        z = unpack(f)
    with np.load(path, allow_pickle=False) as f:
        cfg, inp, tape, _ = cp.load_fixture(f)
    pre = {'fp16': 'q16', 'bf16': 'qbf'}[dt]
    z = {k: v for k, v in z.items() if not k.startswith(pre + '/')}
    out, _ = cp.run_oracle_f64(cfg, inp, tape, cfg.get('aug_p', 0.3), isolated=cfg.get('isolated', False),
                               emu16={'fp16': torch.float16, 'bf16': torch.bfloat16}[dt])
    z.update({f'{pre}/{k}': v for k, v in out.items()})
    np.savez_compressed(path, **pack(z))
    print(tag, dt, 'emulation written', flush=True)


def gen_emulated32(tag, k, cache_dir):
    """One sample of an emulated f32 evaluation of train_<tag>.npz (oracle.sg2_oracle.EMU16 = float32 with
    EMU_JITTER seeded k: every block tensor and gradient rounded to f32 after a random sub-ulp nudge), saved to
    <cache_dir>/e32_<tag>_<k>.npz; emu32merge folds the samples into the fixture as 'e32_<k>/...'.  How far these
    land from the float64 answer is how far f32 rounding ALONE can move a result -- including the discrete
    events (an lrelu mask at a few pixels) that a nudge of the state does not reproduce."""
    import config_parity as cp
    from oracle import sg2_oracle as O
    path = os.path.join(OUT, f'train_{tag}.npz')
    with np.load(path, allow_pickle=False) as f:
        cfg, inp, tape, _ = cp.load_fixture(f)
    O.EMU_JITTER = np.random.default_rng(1000 + int(k))
    try:
        out, _ = cp.run_oracle_f64(cfg, inp, tape, cfg.get('aug_p', 0.3), isolated=cfg.get('isolated', False),
                                   emu16=torch.float32)
    finally:
        O.EMU_JITTER = None
    os.makedirs(cache_dir, exist_ok=True)
    np.savez_compressed(os.path.join(cache_dir, f'e32_{tag}_{k}.npz'), **pack(out))
    print(tag, k, 'f32 emulation sample written', flush=True)


def merge_emulated32(tag, cache_dir):
    from golden_init import unpack
    import glob
    path = os.path.join(OUT, f'train_{tag}.npz')
    with np.load(path, allow_pickle=False) as f:
        z = unpack(f)
    z = {k: v for k, v in z.items() if not k.startswith('e32_')}
    n = 0
    for fn in sorted(glob.glob(os.path.join(cache_dir, f'e32_{tag}_*.npz'))):
        k = fn.rsplit('_', 1)[1][:-4]
        with np.load(fn, allow_pickle=False) as f:
            z.update({f'e32_{k}/{kk}': v for kk, v in unpack(f).items()})
        n += 1
    np.savez_compressed(path, **pack(z))
    print(tag, n, 'f32 emulation samples merged', flush=True)


if __name__ == '__main__':
    which = sys.argv[1:] or ['ops', 'nets'] + list(CONFIGS)
    for tag in CONFIGS:
        if tag in which:
            gen_config_iteration(tag, CONFIGS[tag])
    for tag, base in P0_CONFIGS.items():
        if tag in which:
            gen_config_iteration(tag, CONFIGS[base], aug_p=0.0)
    for w in which:
        if w.startswith('iso:'):           # iso:<tag>[:<batch>]  phase-isolated fixture train_<tag>_iso.npz
            parts = w.split(':')
            base = parts[1][:-2] if parts[1].endswith('p0') else parts[1]
            cfg_i = dict(CONFIGS[base], **({'batch': int(parts[2])} if len(parts) > 2 else {}))
            gen_config_iteration(parts[1], cfg_i, aug_p=0.0 if parts[1].endswith('p0') else 0.3, isolated=True)
        if w.startswith('emu:'):           # emu:<tag>:<fp16|bf16>
            parts = w.split(':')
            gen_emulated16(parts[1], parts[2])
        if w.startswith('emu16n:'):        # emu16n:<tag>:<fp16|bf16>:<seed>   (to $GOLD_CACHE)
            parts = w.split(':')
            gen_emulated16_nudged(parts[1], parts[2], parts[3], os.environ.get('GOLD_CACHE', '/tmp/gold'))
        if w.startswith('emu16p:'):        # emu16p:<tag>:<fp16,bf16>:<seed>[:<k, default 12>]   (to $GOLD_CACHE)
            parts = w.split(':')
            gen_emulated16_perturbed(parts[1], parts[2].split(','), parts[3], int(parts[4]) if len(parts) > 4 else 12,
                                     os.environ.get('GOLD_CACHE', '/tmp/gold'))
        if w.startswith('emu16pmerge:'):   # emu16pmerge:<tag>
            merge_emulated16_perturbed(w.split(':')[1], os.environ.get('GOLD_CACHE', '/tmp/gold'))
        if w.startswith('emu16nmerge:'):   # emu16nmerge:<tag>
            merge_emulated16_nudged(w.split(':')[1], os.environ.get('GOLD_CACHE', '/tmp/gold'))
        if w.startswith('emu32:'):         # emu32:<tag>:<sample k>   (to $GOLD_CACHE, default /tmp/gold)
            parts = w.split(':')
            gen_emulated32(parts[1], parts[2], os.environ.get('GOLD_CACHE', '/tmp/gold'))
        if w.startswith('emu32merge:'):    # emu32merge:<tag>
            merge_emulated32(w.split(':')[1], os.environ.get('GOLD_CACHE', '/tmp/gold'))
        if w.startswith('cond:'):          # cond:<tag>[:<log2 of the nudge, default -24>]
            parts = w.split(':')
            gen_conditioning(parts[1], perturb=2.0 ** float(parts[2]) if len(parts) > 2 else 2.0 ** -24)
    if 'aug' in which:
        gen_augment()
    if 'ops' not in which:
        sys.exit(0)
    gen_upfirdn2d()
    gen_bias_act()
    gen_conv()
    gen_augment()
    if 'nets' in which:
        gen_network(c_dim=2, img_channels=1, tag='claro')
        gen_network(c_dim=0, img_channels=2, tag='pelvis')
    for f in sorted(os.listdir(OUT)):
        if f.endswith('.npz'):
            print(f, os.path.getsize(os.path.join(OUT, f)))
