"""a * b + c with reduced-broadcast gradients (SG3/torch_utils/ops/fma.py:15-58).

Used for the demodulation + noise epilogue of the modulated convolution
(networks_stylegan2.py:71-72)."""
import torch

from .staged_sum import staged_sum


def fma(a, b, c):  # => a * b + c
    return _FMA.apply(a, b, c)


def _sum_to(x, shape):
    """Sum a broadcast gradient back to `shape`."""
    lead = x.ndim - len(shape)
    assert lead >= 0
    dims = [d for d in range(x.ndim) if x.shape[d] > 1 and (d < lead or shape[d - lead] == 1)]
    if dims:
        x = staged_sum(x, dims, keepdim=True)
    if lead:
        x = x.reshape(-1, *x.shape[lead + 1:])
    assert tuple(x.shape) == tuple(shape)
    return x


class _FMA(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, c):
        ctx.save_for_backward(a, b)
        ctx.c_shape = c.shape
        return torch.addcmul(c, a, b)

    @staticmethod
    def backward(ctx, dout):
        a, b = ctx.saved_tensors
        da = _sum_to(dout * b, a.shape) if ctx.needs_input_grad[0] else None
        db = _sum_to(dout * a, b.shape) if ctx.needs_input_grad[1] else None
        dc = _sum_to(dout, ctx.c_shape) if ctx.needs_input_grad[2] else None
        return da, db, dc
