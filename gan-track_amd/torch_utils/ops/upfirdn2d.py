"""upfirdn2d on MI355X (HIP kernel sg2_upfirdn2d, filter taps staged in LDS).

Drop-in for SG3/torch_utils/ops/upfirdn2d.py: `setup_filter`, `upfirdn2d`, `filter2d`,
`upsample2d`, `downsample2d` with identical arguments and padding algebra (:70-389).  Gradients
of any order w.r.t. x (the op is linear; its adjoint is again an upfirdn2d with up/down swapped
and the filter flipped, reference :250-269).  Separable (1-D) filters run as a horizontal then a
vertical pass, like the reference plugin (:243-245).
"""
import ctypes

import numpy as np
import torch

import sg2hip as _hip


def _parse_scaling(scaling):
    if isinstance(scaling, int):
        scaling = [scaling, scaling]
    assert isinstance(scaling, (list, tuple)) and all(isinstance(v, int) for v in scaling)
    sx, sy = scaling
    assert sx >= 1 and sy >= 1
    return sx, sy


def _parse_padding(padding):
    if isinstance(padding, int):
        padding = [padding, padding]
    assert isinstance(padding, (list, tuple)) and all(isinstance(v, int) for v in padding)
    if len(padding) == 2:
        px, py = padding
        padding = [px, px, py, py]
    px0, px1, py0, py1 = padding
    return px0, px1, py0, py1


def _get_filter_size(f):
    if f is None:
        return 1, 1
    assert isinstance(f, torch.Tensor) and f.ndim in [1, 2]
    fw = int(f.shape[-1])
    fh = int(f.shape[0])
    assert fw >= 1 and fh >= 1
    return fw, fh


def setup_filter(f, device=torch.device('cpu'), normalize=True, flip_filter=False, gain=1, separable=None):
    """Prepare a float32 FIR filter (reference :70-114)."""
    if f is None:
        f = 1
    f = torch.as_tensor(f, dtype=torch.float32)
    assert f.ndim in [0, 1, 2] and f.numel() > 0
    if f.ndim == 0:
        f = f[np.newaxis]
    if separable is None:
        separable = (f.ndim == 1 and f.numel() >= 8)
    if f.ndim == 1 and not separable:
        f = f.ger(f)
    assert f.ndim == (1 if separable else 2)
    if normalize:
        f /= f.sum()
    if flip_filter:
        f = f.flip(list(range(f.ndim)))
    f = f * (gain ** (f.ndim / 2))
    return f.to(device=device)


def _raw(x, f2, upx, upy, downx, downy, px0, px1, py0, py1, flip, gain):
    """One sg2_upfirdn2d launch with a 2-D float32 filter f2 [fh, fw]."""
    n, c, h, w = x.shape
    fh, fw = f2.shape
    oh = (h * upy + py0 + py1 - fh + downy) // downy
    ow = (w * upx + px0 + px1 - fw + downx) // downx
    assert oh >= 1 and ow >= 1, 'upfirdn2d: output would be empty'
    fmt = torch.channels_last if (x.stride(1) == 1 and c > 1) else torch.contiguous_format
    y = torch.empty([n, c, oh, ow], dtype=x.dtype, device=x.device, memory_format=fmt)
    _hip.check(_hip.lib().sg2_upfirdn2d(
        _hip.ptr(y), _hip.ptr(x), _hip.ptr(f2), _hip.dtype_code(x), _hip.i64arr(x.shape), _hip.i64arr(x.stride()),
        _hip.i64arr(y.shape), _hip.i64arr(y.stride()), fw, fh, upx, upy, downx, downy, px0, px1, py0, py1,
        int(bool(flip)), float(gain), _hip.stream_ptr(x.device)), 'sg2_upfirdn2d')
    return y


def _raw_lim(x, f2, upx, upy, downx, downy, px0, px1, py0, py1, flip, gain, lim):
    """sg2_upfirdn2d_lim: outputs beyond the device extent `lim` (int32 [2]) are zero-banded / skipped."""
    n, c, h, w = x.shape
    fh, fw = f2.shape
    oh = (h * upy + py0 + py1 - fh + downy) // downy
    ow = (w * upx + px0 + px1 - fw + downx) // downx
    y = torch.empty([n, c, oh, ow], dtype=x.dtype, device=x.device)
    _hip.check(_hip.lib().sg2_upfirdn2d_lim(
        _hip.ptr(y), _hip.ptr(x), _hip.ptr(f2), _hip.dtype_code(x), _hip.i64arr(x.shape), _hip.i64arr(x.stride()),
        _hip.i64arr(y.shape), _hip.i64arr(y.stride()), fw, fh, upx, upy, downx, downy, px0, px1, py0, py1,
        int(bool(flip)), float(gain), _hip.ptr(lim), _hip.stream_ptr(x.device)), 'sg2_upfirdn2d_lim')
    return y


class _SepLimited(torch.autograd.Function):
    """Separable upfirdn2d of a dynamically sized image held in a static buffer (the ADA pipe,
    augment_mi.py): the horizontal pass computes outputs inside extent lims[0], the vertical pass inside
    lims[1]; the backward (the adjoint, again separable) uses lims[2], lims[3], and its own backward the
    forward's.  Exact wherever a consumer reads (see UpfParams::lim in upfirdn2d.hip)."""

    @staticmethod
    def forward(ctx, x, f, up, down, padding, flip_filter, gain, lims):
        upx, upy = up
        downx, downy = down
        px0, px1, py0, py1 = padding
        x = x.contiguous()
        y = _raw_lim(x, f.unsqueeze(0), upx, 1, downx, 1, px0, px1, 0, 0, flip_filter, 1.0, lims[0])
        y = _raw_lim(y, f.unsqueeze(1), 1, upy, 1, downy, 0, 0, py0, py1, flip_filter, gain, lims[1])
        ctx.save_for_backward(f)
        ctx.cfg = (up, down, padding, flip_filter, gain, lims, x.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        f, = ctx.saved_tensors
        up, down, padding, flip_filter, gain, lims, xs = ctx.cfg
        aup, adown, p, aflip = adjoint_params(f, (xs[2], xs[3]), (dy.shape[2], dy.shape[3]), list(up), list(down),
                                              list(padding), flip_filter)
        dx = _SepLimited.apply(dy, f, tuple(aup), tuple(adown), tuple(p), aflip, gain,
                               (lims[2], lims[3], lims[0], lims[1]))
        return dx, None, None, None, None, None, None, None


def upsample2d_limited(x, f, lims, up=2, gain=1):
    """upsample2d (1-D separable filter, f32 NCHW) computing only inside device extents `lims` (four
    int32 [2] tensors: forward horizontal / vertical pass, backward horizontal / vertical pass)."""
    _hip.require_device(x)
    assert f.ndim == 1 and x.dtype == torch.float32
    fw = f.shape[0]
    p = [(fw + up - 1) // 2, (fw - up) // 2] * 2
    return _SepLimited.apply(x, f.to(device=x.device, dtype=torch.float32).contiguous(), (up, up), (1, 1),
                             tuple(p), False, float(gain * up * up), tuple(lims))


def fir_fused(x, f2, padding, gain=1.0, flip_filter=False, out_scale=None, noise=None, noise_gain=1.0, bias=None,
              act=0, alpha=0.2, act_gain=1.0, clamp=-1.0, aux_mode=0):
    """2-D FIR (up = down = 1) with the fused layer epilogue (sg2_upfirdn2d_fused):
    c = FIR(x) * gain;  y = clamp(act(c * out_scale[n,c] + noise * g + bias) * act_gain).
    x NHWC (channels_last) with C % 8 == 0.  Returns (y, aux) with aux = c (aux_mode 1) / y (2)."""
    px0, px1, py0, py1 = _parse_padding(padding)
    n, c, h, w = x.shape
    fh, fw = f2.shape
    oh, ow = h + py0 + py1 - fh + 1, w + px0 + px1 - fw + 1
    y = torch.empty([n, c, oh, ow], dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    aux = torch.empty_like(y) if aux_mode else None
    epi = _hip.Epilogue(_hip.ptr(out_scale), _hip.ptr(noise), _hip.ptr(bias), None, _hip.ptr(aux), float(noise_gain),
                        float(alpha), float(act_gain), float(clamp), int(act), int(aux_mode))
    _hip.check(_hip.lib().sg2_upfirdn2d_fused(
        _hip.ptr(y), _hip.ptr(x), _hip.ptr(f2), _hip.dtype_code(x), _hip.i64arr(x.shape), _hip.i64arr(x.stride()),
        _hip.i64arr(y.shape), _hip.i64arr(y.stride()), fw, fh, 1, 1, 1, 1, px0, px1, py0, py1, int(bool(flip_filter)),
        float(gain), ctypes.byref(epi), _hip.stream_ptr(x.device)), 'sg2_upfirdn2d_fused')
    return y, aux


class _ForkFIR(torch.autograd.Function):
    """(x, upfirdn2d(x, f, down=down, padding)) for a tensor that feeds both a FIR-downsampled branch and an
    unfiltered one (DiscriminatorBlock's resnet skip and conv0, networks_stylegan2.py:621-627).  The
    backward fuses the add of the two branch gradients into the adjoint FIR (its epilogue's residual
    term): dx = round(FIR^T(g_down)) + g_x, the sum autograd would form, without an activation-sized add
    pass.  Under create_graph the same gradient is built from differentiable ops."""

    @staticmethod
    def forward(ctx, x, f, down, padding):
        px0, px1, py0, py1 = padding
        y = _raw(x, f, 1, 1, down, down, px0, px1, py0, py1, False, 1.0)
        ctx.save_for_backward(f)
        ctx.cfg = (down, padding, x.shape)
        return x.view_as(x), y

    @staticmethod
    def backward(ctx, gx, gy):
        f, = ctx.saved_tensors
        down, padding, xs = ctx.cfg
        if gy is None:
            return gx, None, None, None
        aup, adown, p, aflip = adjoint_params(f, (xs[2], xs[3]), (gy.shape[2], gy.shape[3]), [1, 1], [down, down],
                                              list(padding), False)
        if torch.is_grad_enabled() or gx is None:
            dx = _upfirdn2d_fn(up=aup, down=adown, padding=p, flip_filter=aflip).apply(gy, f)
            return (dx + gx if gx is not None else dx), None, None, None
        cl = torch.channels_last
        gy = gy.contiguous(memory_format=cl)
        gx = gx.to(gy.dtype).contiguous(memory_format=cl)
        dx = torch.empty_like(gx)
        epi = _hip.Epilogue(None, None, None, _hip.ptr(gx), None, 1.0, 0.2, 1.0, -1.0, 0, 0)
        fh, fw = f.shape
        _hip.check(_hip.lib().sg2_upfirdn2d_fused(
            _hip.ptr(dx), _hip.ptr(gy), _hip.ptr(f), _hip.dtype_code(gy), _hip.i64arr(gy.shape),
            _hip.i64arr(gy.stride()), _hip.i64arr(dx.shape), _hip.i64arr(dx.stride()), fw, fh, aup[0], aup[1],
            adown[0], adown[1], p[0], p[1], p[2], p[3], int(bool(aflip)), 1.0, ctypes.byref(epi),
            _hip.stream_ptr(gy.device)), 'sg2_upfirdn2d_fused')
        return dx, None, None, None


def fork_fir(x, f, down, padding):
    """(x, upfirdn2d(x, f, down=down, padding=padding)) with the branch-gradient add fused into the
    backward (_ForkFIR).  f: a 2-D float32 filter on x's device; x channels-last with C % 8 == 0 (16-bit)
    or C % 4 == 0 (f32), as the fused epilogue requires."""
    _hip.require_device(x)
    px0, px1, py0, py1 = _parse_padding(padding)
    f = f.to(device=x.device, dtype=torch.float32).contiguous()
    return _ForkFIR.apply(x, f, int(down), (px0, px1, py0, py1))


def fork_fir_ok(x, f):
    """Whether fork_fir's fused backward applies (else the caller runs the plain two-branch graph)."""
    v = 8 if x.dtype in (torch.float16, torch.bfloat16) else 4
    return (x.is_cuda and f is not None and f.ndim == 2 and x.ndim == 4 and x.shape[1] % v == 0 and
            x.is_contiguous(memory_format=torch.channels_last))


def adjoint_params(f, x_hw, y_hw, up, down, padding, flip_filter):
    """(up, down, padding, flip) of the adjoint upfirdn2d (reference upfirdn2d.py:250-269)."""
    upx, upy = _parse_scaling(up)
    downx, downy = _parse_scaling(down)
    px0, px1, py0, py1 = _parse_padding(padding)
    fw, fh = _get_filter_size(f)
    ih, iw = x_hw
    oh, ow = y_hw
    p = [fw - px0 - 1, iw * upx - ow * downx + px0 - upx + 1, fh - py0 - 1, ih * upy - oh * downy + py0 - upy + 1]
    return [downx, downy], [upx, upy], p, not flip_filter


_cache = {}


def _upfirdn2d_fn(up=1, down=1, padding=0, flip_filter=False, gain=1):
    upx, upy = _parse_scaling(up)
    downx, downy = _parse_scaling(down)
    px0, px1, py0, py1 = _parse_padding(padding)
    key = (upx, upy, downx, downy, px0, px1, py0, py1, flip_filter, gain)
    if key in _cache:
        return _cache[key]

    class Upfirdn2d(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, f):
            assert x.ndim == 4
            if f is None:
                f = torch.ones([1, 1], dtype=torch.float32, device=x.device)
            if f.ndim == 1 and f.shape[0] == 1:
                f = f.square().unsqueeze(0)
            f = f.to(device=x.device, dtype=torch.float32).contiguous()
            if f.ndim == 2:
                y = _raw(x, f, upx, upy, downx, downy, px0, px1, py0, py1, flip_filter, gain)
            else:
                y = _raw(x, f.unsqueeze(0), upx, 1, downx, 1, px0, px1, 0, 0, flip_filter, 1.0)
                y = _raw(y, f.unsqueeze(1), 1, upy, 1, downy, 0, 0, py0, py1, flip_filter, gain)
            ctx.save_for_backward(f)
            ctx.x_shape = x.shape
            return y

        @staticmethod
        def backward(ctx, dy):
            f, = ctx.saved_tensors
            _, _, ih, iw = ctx.x_shape
            _, _, oh, ow = dy.shape
            # adjoint: upsample by `down`, filter with the flipped taps, decimate by `up`
            aup, adown, p, aflip = adjoint_params(f, (ih, iw), (oh, ow), [upx, upy], [downx, downy],
                                                  [px0, px1, py0, py1], flip_filter)
            dx = None
            if ctx.needs_input_grad[0]:
                dx = _upfirdn2d_fn(up=aup, down=adown, padding=p, flip_filter=aflip, gain=gain).apply(dy, f)
            assert not ctx.needs_input_grad[1]
            return dx, None

    _cache[key] = Upfirdn2d
    return Upfirdn2d


def upfirdn2d(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1, impl='cuda'):
    """Pad, upsample, filter and downsample a batch of 2-D images (reference :118-162)."""
    assert isinstance(x, torch.Tensor)
    _hip.require_device(x)
    return _upfirdn2d_fn(up=up, down=down, padding=padding, flip_filter=flip_filter, gain=gain).apply(x, f)


def filter2d(x, f, padding=0, flip_filter=False, gain=1, impl='cuda'):
    """Filter keeping the input size (reference :277-309)."""
    px0, px1, py0, py1 = _parse_padding(padding)
    fw, fh = _get_filter_size(f)
    p = [px0 + fw // 2, px1 + (fw - 1) // 2, py0 + fh // 2, py1 + (fh - 1) // 2]
    return upfirdn2d(x, f, padding=p, flip_filter=flip_filter, gain=gain, impl=impl)


def upsample2d(x, f, up=2, padding=0, flip_filter=False, gain=1, impl='cuda'):
    """Upsample by `up` (reference :313-348)."""
    upx, upy = _parse_scaling(up)
    px0, px1, py0, py1 = _parse_padding(padding)
    fw, fh = _get_filter_size(f)
    p = [px0 + (fw + upx - 1) // 2, px1 + (fw - upx) // 2, py0 + (fh + upy - 1) // 2, py1 + (fh - upy) // 2]
    return upfirdn2d(x, f, up=up, padding=p, flip_filter=flip_filter, gain=gain * upx * upy, impl=impl)


def downsample2d(x, f, down=2, padding=0, flip_filter=False, gain=1, impl='cuda'):
    """Downsample by `down` (reference :352-387)."""
    downx, downy = _parse_scaling(down)
    px0, px1, py0, py1 = _parse_padding(padding)
    fw, fh = _get_filter_size(f)
    p = [px0 + (fw - downx + 1) // 2, px1 + (fw - downx) // 2, py0 + (fh - downy + 1) // 2, py1 + (fh - downy) // 2]
    return upfirdn2d(x, f, down=down, padding=p, flip_filter=flip_filter, gain=gain, impl=impl)
