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


def affine_grid_sample(input, theta, size, dyn_hw=None):
    """grid_sample(input, affine_grid(theta, size, align_corners=False)) with the grid built inside the
    kernel (sg2_affine_grid_sample_fwd/_bwd) instead of materialised in HBM: the ADA geometric step,
    SG3/training/augment_mi.py:317-318.  theta float [N, 2, 3] (no gradient); size = [N, C, Ho, Wo]."""
    _hip.require_device(input, theta)
    assert theta.shape == (size[0], 2, 3) and input.shape[:2] == tuple(size[:2])
    return _Fwd.apply(input, theta.float().contiguous(), dyn_hw, tuple(size[2:]))


def _sizes(inp, out):
    return (_hip.i64arr(inp.shape), _hip.i64arr(inp.stride()), _hip.i64arr(out.shape), _hip.i64arr(out.stride()))


class _Fwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inp, g, dyn_hw, affine_hw=None):
        """g: grid [N, Ho, Wo, 2], or theta [N, 2, 3] with affine_hw = (Ho, Wo)."""
        n, c = inp.shape[:2]
        if affine_hw is None:
            assert inp.ndim == 4 and g.ndim == 4 and g.shape[-1] == 2
            g = g.float().contiguous()
            ho, wo = g.shape[1], g.shape[2]
        else:
            ho, wo = affine_hw
        out = torch.empty([n, c, ho, wo], dtype=inp.dtype, device=inp.device)
        fn = 'sg2_grid_sample_fwd' if affine_hw is None else 'sg2_affine_grid_sample_fwd'
        _hip.check(getattr(_hip.lib(), fn)(_hip.ptr(out), _hip.ptr(inp), _hip.ptr(g), _hip.dtype_code(inp),
                                           *_sizes(inp, out), _hip.ptr(dyn_hw), _hip.stream_ptr(inp.device)), fn)
        ctx.save_for_backward(inp, g, dyn_hw)
        ctx.affine_hw = affine_hw
        return out

    @staticmethod
    def backward(ctx, gout):
        inp, g, dyn_hw = ctx.saved_tensors
        gin = _Bwd.apply(gout, inp, g, dyn_hw, ctx.affine_hw) if ctx.needs_input_grad[0] else None
        assert not ctx.needs_input_grad[1], 'grid gradients are not supported'
        return gin, None, None, None


class _Bwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gout, inp, g, dyn_hw, affine_hw=None):
        gin = torch.empty(inp.shape, dtype=torch.float32, device=inp.device)
        fn = 'sg2_grid_sample_bwd' if affine_hw is None else 'sg2_affine_grid_sample_bwd'
        _hip.check(getattr(_hip.lib(), fn)(_hip.ptr(gin), _hip.ptr(gout), _hip.ptr(g), _hip.dtype_code(gout),
                                           *_sizes(gin, gout), _hip.ptr(dyn_hw), _hip.stream_ptr(gout.device)), fn)
        ctx.save_for_backward(g, dyn_hw)
        ctx.affine_hw = affine_hw
        return gin.to(inp.dtype)

    @staticmethod
    def backward(ctx, ggin):
        g, dyn_hw = ctx.saved_tensors
        ggout = _Fwd.apply(ggin, g, dyn_hw, ctx.affine_hw) if ctx.needs_input_grad[0] else None
        return ggout, None, None, None, None
