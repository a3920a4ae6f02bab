"""Deterministic network states and result summaries for the configuration-width fixtures
(test infrastructure; no dependency on the reference or the product).

Full-width networks (e.g. 64^2 / cbase 16384: ~20M parameters per network) are too large to commit as
fixtures, so both sides derive the same initial state from the parameter NAMES: `init_state` replaces
every tensor the reference's constructors fill randomly (weights, noise_const) by numpy draws keyed by
(seed, name), scaled like the constructor's own init (randn / lr_multiplier: the scale is the power of
ten nearest the constructed tensor's std), and gives constant-initialised biases / noise strengths
non-trivial values so every gradient path carries signal.  Resample filters and w_avg are kept.

`summarize` reduces a named set of tensors to what a fixture stores: the float64 L2 norm and values at
8 fixed positions (a function of the name) per tensor.
"""
import zlib

import numpy as np
import torch

N_SAMPLES = 8


def _rs(seed, name):
    return np.random.RandomState((zlib.crc32(name.encode()) + 7919 * seed) % (2 ** 32))


def init_state(module, seed=0):
    named = list(module.named_parameters()) + list(module.named_buffers())
    with torch.no_grad():
        for name, t in named:
            if not t.is_floating_point() or 'resample_filter' in name or name.endswith('w_avg') or t.numel() == 0:
                continue
            r = _rs(seed, name)
            if name.endswith('noise_strength'):
                v = np.full(tuple(t.shape), 0.1)
            elif name.endswith('bias') or name.endswith('bias_gain'):
                base = float(t.flatten()[0])          # constructor constant (0, or 1 for affine / bias_init)
                v = base + 0.1 * r.standard_normal(tuple(t.shape))
            else:
                std = float(t.float().std()) if t.numel() > 1 else 1.0
                scale = 10.0 ** round(np.log10(std)) if std > 0 else 1.0
                v = scale * r.standard_normal(tuple(t.shape))
            t.copy_(torch.from_numpy(v.astype(np.float32)).to(t.dtype).to(t.device))


def sample_index(name, numel):
    return _rs(0, name).randint(0, numel, size=min(N_SAMPLES, numel))


def summarize(named, prefix):
    """{name: tensor} -> {prefix/name/norm: f64, prefix/name/numel, prefix/name/samples: f32[<=8]}"""
    out = {}
    for name, t in named.items():
        f = t.detach().double().cpu().flatten()
        out[f'{prefix}/{name}/norm'] = np.array(float(f.norm()), np.float64)
        out[f'{prefix}/{name}/numel'] = np.array(f.numel(), np.int64)
        out[f'{prefix}/{name}/samples'] = f[torch.from_numpy(sample_index(name, f.numel()))].numpy().astype(np.float32)
    return out


def pack(d):
    """Store a summarize()-style dict compactly: the per-tensor entries of every group become four arrays
    (names, norms, element counts, samples padded with NaN); other keys pass through."""
    out, names = {}, []
    for k in d:
        if k.endswith('/norm'):
            names.append(k[:-5])
        elif not (k.endswith('/numel') or k.endswith('/samples')):
            out[k] = d[k]
    out['summ__names'] = np.array(names)
    out['summ__norm'] = np.array([float(d[n + '/norm']) for n in names], np.float64)
    out['summ__numel'] = np.array([int(d[n + '/numel']) for n in names], np.int64)
    smp = np.full([len(names), N_SAMPLES], np.nan, np.float32)
    for i, n in enumerate(names):
        v = np.asarray(d[n + '/samples'])
        smp[i, :v.size] = v
    out['summ__samples'] = smp
    return out


def unpack(z):
    """Inverse of pack (accepts an NpzFile or a dict)."""
    d = {k: z[k] for k in z if not k.startswith('summ__')}
    if 'summ__names' in z:
        # each array read once (an NpzFile decompresses the whole member on every z[key])
        numel, norm, samples = z['summ__numel'], z['summ__norm'], z['summ__samples']
        for i, n in enumerate(z['summ__names'].tolist()):
            d[n + '/norm'] = norm[i]
            d[n + '/numel'] = numel[i]
            d[n + '/samples'] = samples[i, :min(N_SAMPLES, int(numel[i]))]
    return d
