"""Deterministic random-number tape for golden-vector parity (test infrastructure).

The reference draws noise, z, style-mixing cutoffs and ADA parameters from torch's
global RNG (e.g. SG3/training/networks_stylegan2.py:317, SG3/training/loss.py:47-49,89,
SG3/training/augment_mi.py:214-279).  CPU and GPU generators differ, so parity runs
record every draw on the reference side (``Tape.record``) and replay the same arrays,
in the same order, on our side (``Tape.replay``).  Draws are plain numpy arrays so the
tape can be saved in an ``.npz`` fixture.

This module has no dependency on the reference or on the product package.
"""
import contextlib

import numpy as np
import torch


def _shape(args, kwargs):
    if 'size' in kwargs:
        s = kwargs['size']
    elif len(args) == 1 and isinstance(args[0], (list, tuple, torch.Size)):
        s = args[0]
    else:
        s = args
    return tuple(int(v) for v in s)


class Tape:
    def __init__(self, seed=1234, entries=None):
        self.seed = seed
        self.rs = np.random.RandomState(seed)
        self.entries = [] if entries is None else list(entries)
        self.bounds = []      # (lo, hi) of every randint draw, in order (for the compact form)
        self.pos = 0
        self.mode = None

    # --- serialisation -----------------------------------------------------
    def to_npz_dict(self, prefix='tape'):
        d = {f'{prefix}_n': np.array(len(self.entries))}
        for i, (kind, arr) in enumerate(self.entries):
            d[f'{prefix}_{i}_kind'] = np.array(kind)
            d[f'{prefix}_{i}_val'] = arr
        return d

    def to_compact_npz_dict(self, prefix='tape'):
        """Seed + the (kind, shape, bounds) sequence only: the values are regenerated from the seed on
        load (the recording draws them from one numpy RandomState in this order)."""
        kinds = np.array([k for k, _ in self.entries])
        shapes = np.array(repr([tuple(a.shape) for _, a in self.entries]))
        return {f'{prefix}_seed': np.array(self.seed), f'{prefix}_kinds': kinds, f'{prefix}_shapes': shapes,
                f'{prefix}_bounds': np.array(self.bounds, dtype=np.int64).reshape(-1, 2)}

    @classmethod
    def from_npz(cls, z, prefix='tape'):
        if f'{prefix}_seed' in z:
            import ast
            t = cls(seed=int(z[f'{prefix}_seed']))
            t.mode = 'record'
            bounds = iter(z[f'{prefix}_bounds'].tolist())
            for kind, shape in zip(z[f'{prefix}_kinds'].tolist(), ast.literal_eval(str(z[f'{prefix}_shapes']))):
                lo, hi = next(bounds) if kind == 'randint' else (None, None)
                t._draw(str(kind), tuple(shape), lo, hi)
            t.mode = None
            return t
        n = int(z[f'{prefix}_n'])
        ents = [(str(z[f'{prefix}_{i}_kind']), z[f'{prefix}_{i}_val']) for i in range(n)]
        return cls(entries=ents)

    # --- draw --------------------------------------------------------------
    def _draw(self, kind, shape, lo=None, hi=None):
        if self.mode == 'record':
            if kind == 'randn':
                arr = self.rs.standard_normal(shape).astype(np.float32)
            elif kind == 'rand':
                arr = self.rs.random_sample(shape).astype(np.float32)
            else:
                arr = np.array(self.rs.randint(lo, hi), dtype=np.int64)
                self.bounds.append((lo, hi))
            self.entries.append((kind, arr))
            return arr
        kind0, arr = self.entries[self.pos]
        self.pos += 1
        if kind0 != kind or tuple(arr.shape) != tuple(shape):
            raise RuntimeError(f'RNG tape mismatch at draw {self.pos - 1}: tape has {kind0}{tuple(arr.shape)}, '
                               f'caller asked for {kind}{tuple(shape)}')
        return arr

    def _mk(self, kind, shape, dtype=None, device=None):
        arr = self._draw(kind, shape)
        t = torch.from_numpy(np.array(arr))
        if dtype is None and t.is_floating_point():
            dtype = torch.get_default_dtype()      # as torch.randn / torch.rand without a dtype
        if dtype is not None:
            t = t.to(dtype)
        if device is not None:
            t = t.to(device)
        return t

    @contextlib.contextmanager
    def _patched(self, mode):
        self.mode = mode
        orig = (torch.randn, torch.rand, torch.randn_like, torch.rand_like, torch.Tensor.random_)
        tape = self

        def randn(*args, **kw):
            return tape._mk('randn', _shape(args, kw), kw.get('dtype'), kw.get('device'))

        def rand(*args, **kw):
            return tape._mk('rand', _shape(args, kw), kw.get('dtype'), kw.get('device'))

        def randn_like(t, **kw):
            return tape._mk('randn', tuple(t.shape), kw.get('dtype', t.dtype), kw.get('device', t.device))

        def rand_like(t, **kw):
            return tape._mk('rand', tuple(t.shape), kw.get('dtype', t.dtype), kw.get('device', t.device))

        def random_(self_t, lo=0, hi=None, **kw):
            if hi is None:
                lo, hi = 0, lo
            v = tape._draw('randint', (), lo, hi)
            with torch.no_grad():
                self_t.fill_(int(v))
            return self_t

        torch.randn, torch.rand, torch.randn_like, torch.rand_like = randn, rand, randn_like, rand_like
        torch.Tensor.random_ = random_
        try:
            yield self
        finally:
            torch.randn, torch.rand, torch.randn_like, torch.rand_like, torch.Tensor.random_ = orig
            self.mode = None

    def record(self):
        return self._patched('record')

    def replay(self):
        self.pos = 0
        return self._patched('replay')
