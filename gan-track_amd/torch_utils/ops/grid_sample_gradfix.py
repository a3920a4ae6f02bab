"""Bilinear grid_sample with gradients of arbitrary order w.r.t. the input, on the HIP kernels
sg2_grid_sample_fwd / sg2_grid_sample_bwd.

Drop-in for SG3/torch_utils/ops/grid_sample_gradfix.py:28-83 (mode='bilinear',
padding_mode='zeros', align_corners=False; the grid gets no gradient, as on the reference's
training path where it is built from random augmentation parameters)."""
import torch

import sg2hip as _hip

enabled = True


def grid_sample(input, grid, dyn_hw=None):
    """dyn_hw (extension, optional): device int32 [2] logical input size when `input` is a larger static
    buffer holding the image at its origin (the ADA pipe's sync-free padding)."""
    _hip.require_device(input, grid)
    return _Fwd.apply(input, grid, dyn_hw)


def _sizes(inp, out):
    return (_hip.i64arr(inp.shape), _hip.i64arr(inp.stride()), _hip.i64arr(out.shape), _hip.i64arr(out.stride()))


class _Fwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inp, grid, dyn_hw):
        assert inp.ndim == 4 and grid.ndim == 4 and grid.shape[-1] == 2
        g = grid.float().contiguous()
        n, c = inp.shape[:2]
        out = torch.empty([n, c, g.shape[1], g.shape[2]], dtype=inp.dtype, device=inp.device)
        _hip.check(_hip.lib().sg2_grid_sample_fwd(_hip.ptr(out), _hip.ptr(inp), _hip.ptr(g), _hip.dtype_code(inp),
                                                  *_sizes(inp, out), _hip.ptr(dyn_hw), _hip.stream_ptr(inp.device)),
                   'sg2_grid_sample_fwd')
        ctx.save_for_backward(inp, g, dyn_hw)
        return out

    @staticmethod
    def backward(ctx, gout):
        inp, g, dyn_hw = ctx.saved_tensors
        gin = _Bwd.apply(gout, inp, g, dyn_hw) if ctx.needs_input_grad[0] else None
        assert not ctx.needs_input_grad[1], 'grid gradients are not supported'
        return gin, None, None


class _Bwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gout, inp, g, dyn_hw):
        gin = torch.empty(inp.shape, dtype=torch.float32, device=inp.device)
        _hip.check(_hip.lib().sg2_grid_sample_bwd(_hip.ptr(gin), _hip.ptr(gout), _hip.ptr(g), _hip.dtype_code(gout),
                                                  *_sizes(gin, gout), _hip.ptr(dyn_hw), _hip.stream_ptr(gout.device)),
                   'sg2_grid_sample_bwd')
        ctx.save_for_backward(g, dyn_hw)
        return gin.to(inp.dtype)

    @staticmethod
    def backward(ctx, ggin):
        g, dyn_hw = ctx.saved_tensors
        ggout = _Fwd.apply(ggin, g, dyn_hw) if ctx.needs_input_grad[0] else None
        return ggout, None, None, None
