"""Helpers shared by the golden-vector tests (test infrastructure)."""
import ast
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def lit(z, key):
    return ast.literal_eval(str(z[key]))


def rel_err(a, b):
    a = torch.as_tensor(np.asarray(a, dtype=np.float64)) if not isinstance(a, torch.Tensor) else a.double().cpu()
    b = torch.as_tensor(np.asarray(b, dtype=np.float64)) if not isinstance(b, torch.Tensor) else b.double().cpu()
    assert tuple(a.shape) == tuple(b.shape), (tuple(a.shape), tuple(b.shape))
    den = b.norm().item()
    num = (a - b).norm().item()
    return num / max(den, 1e-30)


def load_state(module, z, prefix):
    """Copy '<prefix>/<name>' arrays of a golden npz into module params/buffers."""
    named = dict(list(module.named_parameters()) + list(module.named_buffers()))
    keys = [k for k in z.files if k.startswith(prefix + '/')]
    assert keys, prefix
    seen = set()
    with torch.no_grad():
        for k in keys:
            n = k[len(prefix) + 1:]
            assert n in named, f'{n} missing in module'
            t = named[n]
            t.copy_(torch.from_numpy(z[k]).to(t.dtype).reshape(t.shape))
            seen.add(n)
    missing = set(named) - seen
    assert not missing, f'golden lacks {sorted(missing)[:5]}'


def compare_state(module, z, prefix, tol, skip=()):
    named = dict(list(module.named_parameters()) + list(module.named_buffers()))
    worst = (0.0, None)
    for n, t in named.items():
        if any(s in n for s in skip):
            continue
        e = rel_err(t.detach().float().cpu(), z[f'{prefix}/{n}'])
        if e > worst[0]:
            worst = (e, n)
        assert e <= tol, f'{prefix}/{n}: rel err {e:.3g} > {tol}'
    return worst
