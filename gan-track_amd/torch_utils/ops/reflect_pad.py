"""Reflect padding with margins held in device memory (HIP kernel sg2_reflect_pad_dyn).

The reference pads the ADA pipe's images by margins computed from the random transforms and read
back to the host (SG3/training/augment_mi.py:295-301: `margin.ceil().to(torch.int32)` unpacked into
Python ints, then `torch.nn.functional.pad(..., mode='reflect')`).  Here the margins stay on the
device: the padded image is written at the origin of a static [N, C, 3H-2, 3W-2] buffer with zeros
elsewhere -- exactly the values upfirdn2d's implicit zero padding sees around the reference's
dynamically sized image -- and the logical size travels to the grid sampler as a device tensor.
No host synchronisation, static shapes: the whole training step can be captured in a HIP graph.
Linear op: the gradient is the adjoint (a gather of the reflected positions), whose gradient is the
forward again, so the R1 double backward works.
"""
import torch

import sg2hip as _hip


def _launch(y, x, margins, n, c, h, w, hs, ws, adjoint):
    _hip.check(_hip.lib().sg2_reflect_pad_dyn(_hip.ptr(y), _hip.ptr(x), _hip.ptr(margins), n, c, h, w, hs, ws,
                                              int(adjoint), _hip.stream_ptr(x.device)), 'sg2_reflect_pad_dyn')
    return y


class _Pad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, margins):
        assert x.dtype == torch.float32 and margins.dtype == torch.int32
        x = x.contiguous()
        n, c, h, w = x.shape
        y = torch.empty([n, c, 3 * h - 2, 3 * w - 2], dtype=x.dtype, device=x.device)
        ctx.save_for_backward(margins)
        ctx.hw = (h, w)
        return _launch(y, x, margins, n, c, h, w, 3 * h - 2, 3 * w - 2, False)

    @staticmethod
    def backward(ctx, gy):
        margins, = ctx.saved_tensors
        h, w = ctx.hw
        gx = _Adj.apply(gy, margins, h, w) if ctx.needs_input_grad[0] else None
        return gx, None


class _Adj(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gy, margins, h, w):
        gy = gy.contiguous()
        n, c, hs, ws = gy.shape
        gx = torch.empty([n, c, h, w], dtype=gy.dtype, device=gy.device)
        ctx.save_for_backward(margins)
        return _launch(gx, gy, margins, n, c, h, w, hs, ws, True)

    @staticmethod
    def backward(ctx, ggx):
        margins, = ctx.saved_tensors
        ggy = _Pad.apply(ggx, margins) if ctx.needs_input_grad[0] else None
        return ggy, None, None, None


def reflect_pad_dyn(x, margins):
    """x [N,C,H,W] f32, margins device int32 [4] = (mx0, my0, mx1, my1), each <= size - 1."""
    _hip.require_device(x, margins)
    return _Pad.apply(x, margins)
