"""Fused bias + activation on MI355X (HIP kernel sg2_bias_act).

Drop-in for SG3/torch_utils/ops/bias_act.py: same `bias_act()` signature, the same
`activation_funcs` table (ids = the reference plugin's cuda_idx, :21-31), first- and second-order
gradients through an explicit grad op (reference :142-203).  There is no slow path: `impl` is
accepted for signature compatibility and ignored; non-device tensors raise.
"""
import numpy as np
import torch

import dnnlib
import sg2hip as _hip

from . import staged_sum

activation_funcs = {
    'linear': dnnlib.EasyDict(def_alpha=0, def_gain=1, cuda_idx=1, ref='', has_2nd_grad=False),
    'relu': dnnlib.EasyDict(def_alpha=0, def_gain=np.sqrt(2), cuda_idx=2, ref='y', has_2nd_grad=False),
    'lrelu': dnnlib.EasyDict(def_alpha=0.2, def_gain=np.sqrt(2), cuda_idx=3, ref='y', has_2nd_grad=False),
    'tanh': dnnlib.EasyDict(def_alpha=0, def_gain=1, cuda_idx=4, ref='y', has_2nd_grad=True),
    'sigmoid': dnnlib.EasyDict(def_alpha=0, def_gain=1, cuda_idx=5, ref='y', has_2nd_grad=True),
    'elu': dnnlib.EasyDict(def_alpha=0, def_gain=1, cuda_idx=6, ref='y', has_2nd_grad=True),
    'selu': dnnlib.EasyDict(def_alpha=0, def_gain=1, cuda_idx=7, ref='y', has_2nd_grad=True),
    'softplus': dnnlib.EasyDict(def_alpha=0, def_gain=1, cuda_idx=8, ref='y', has_2nd_grad=True),
    'swish': dnnlib.EasyDict(def_alpha=0, def_gain=np.sqrt(2), cuda_idx=9, ref='x', has_2nd_grad=True),
}


def _layout(x):
    return torch.channels_last if x.ndim == 4 and x.stride(1) == 1 and x.shape[1] > 1 else torch.contiguous_format


def _dense(t, fmt):
    if t is None:
        return None
    t = t.contiguous(memory_format=fmt) if t.ndim == 4 else t.contiguous()
    if t.data_ptr() % 16:
        t = t.clone(memory_format=fmt) if t.ndim == 4 else t.clone()
    return t


def _launch(x, b, xref, yref, dy, grad, dim, spec, alpha, gain, clamp):
    y = torch.empty_like(x)
    size_b = b.numel() if b is not None else 1
    step_b = x.stride(dim) if b is not None else 1
    _hip.check(_hip.lib().sg2_bias_act(_hip.ptr(y), _hip.ptr(x), _hip.ptr(b), _hip.ptr(xref), _hip.ptr(yref),
                                       _hip.ptr(dy), _hip.dtype_code(x), x.numel(), size_b, step_b, grad,
                                       spec.cuda_idx, alpha, gain, clamp, _hip.stream_ptr(x.device)),
               'sg2_bias_act')
    return y


_cache = {}


def _bias_act_fn(dim, act, alpha, gain, clamp):
    key = (dim, act, alpha, gain, clamp)
    if key in _cache:
        return _cache[key]
    spec = activation_funcs[act]
    trivial = act == 'linear' and gain == 1 and clamp < 0

    class BiasActGrad(torch.autograd.Function):
        """dx = grad(dy; x, b, y)   (reference bias_act.py:175-203)."""

        @staticmethod
        def forward(ctx, dy, x, b, y):
            ref = y if y is not None else x
            fmt = _layout(ref) if ref is not None else _layout(dy)
            dy = _dense(dy, fmt)
            x = _dense(x, fmt)
            y = _dense(y, fmt)
            ctx.fmt = fmt
            dx = _launch(dy, b, x, y, None, 1, dim, spec, alpha, gain, clamp)
            ctx.save_for_backward(dy if spec.has_2nd_grad else None, x, b, y)
            return dx

        @staticmethod
        def backward(ctx, d_dx):
            d_dx = _dense(d_dx, ctx.fmt)
            dy, x, b, y = ctx.saved_tensors
            d_dy = d_x = d_b = None
            if ctx.needs_input_grad[0]:
                d_dy = BiasActGrad.apply(d_dx, x, b, y)
            if spec.has_2nd_grad and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2]):
                d_x = _launch(d_dx, b, x, y, dy, 2, dim, spec, alpha, gain, clamp)
            if spec.has_2nd_grad and ctx.needs_input_grad[2]:
                d_b = staged_sum.staged_sum(d_x, [i for i in range(d_x.ndim) if i != dim])
            return d_dy, d_x, d_b, None

    class BiasAct(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, b):
            fmt = _layout(x)
            x = _dense(x, fmt)
            b = b.contiguous() if b is not None else None
            ctx.fmt = fmt
            y = x if (trivial and b is None) else _launch(x, b, None, None, None, 0, dim, spec, alpha, gain, clamp)
            keep_x = 'x' in spec.ref or spec.has_2nd_grad
            # y is also needed for the clamp mask when clamping is on (the reference's plugin drops it
            # for 'linear', so its GPU gradient ignores the clamp there; its CPU path and this build mask)
            keep_y = 'y' in spec.ref or clamp >= 0
            ctx.save_for_backward(x if keep_x else None, b if keep_x else None, y if keep_y else None)
            return y

        @staticmethod
        def backward(ctx, dy):
            dy = _dense(dy, ctx.fmt)
            x, b, y = ctx.saved_tensors
            dx = db = None
            if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
                dx = dy if trivial else BiasActGrad.apply(dy, x, b, y)
            if ctx.needs_input_grad[1]:
                db = staged_sum.staged_sum(dx, [i for i in range(dx.ndim) if i != dim])
            return dx, db

    BiasAct.Grad = BiasActGrad
    _cache[key] = BiasAct
    return BiasAct


def bias_act_grad(dy, y, act='linear', alpha=None, gain=None, clamp=None, dim=1):
    """Differentiable dL/dx of y = bias_act(x, ...) given dL/dy and the saved output y (for activations
    whose derivative is expressed through y, reference `ref='y'`).  Used by fused layer backwards."""
    spec = activation_funcs[act]
    assert 'x' not in spec.ref
    alpha = float(alpha if alpha is not None else spec.def_alpha)
    gain = float(gain if gain is not None else spec.def_gain)
    clamp = float(clamp if clamp is not None else -1)
    dy = _dense(dy, _layout(y))     # the kernel indexes dy and y with one flat index
    return _bias_act_fn(dim, act, alpha, gain, clamp).Grad.apply(dy, None, None, y)


def bias_act(x, b=None, dim=1, act='linear', alpha=None, gain=None, clamp=None, impl='cuda'):
    """y = clamp(act(x + b) * gain).  See SG3/torch_utils/ops/bias_act.py:52-86."""
    assert isinstance(x, torch.Tensor)
    assert clamp is None or clamp >= 0
    _hip.require_device(x, b)
    spec = activation_funcs[act]
    alpha = float(alpha if alpha is not None else spec.def_alpha)
    gain = float(gain if gain is not None else spec.def_gain)
    clamp = float(clamp if clamp is not None else -1)
    if b is not None:
        assert b.ndim == 1 and b.shape[0] == x.shape[dim] and b.dtype == x.dtype
    return _bias_act_fn(dim, act, alpha, gain, clamp).apply(x, b)
