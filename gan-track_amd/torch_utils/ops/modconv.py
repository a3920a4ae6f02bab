"""Fused StyleGAN2 synthesis layer (3x3, up = 1) on the LDS-halo MFMA kernel (sg2_conv3x3).

Forward, ONE kernel (reference SG3/training/networks_stylegan2.py:309-328 and modulated_conv2d
:32-77, non-fused training form):
    c = conv2d(x * s[n, ci], W)                  (modulation applied while staging x into LDS)
    y = clamp(lrelu(c * d[n, co] + noise + b) * gain, +-clamp)
where the reference runs x*s, conv, fma(x, d, noise) and bias_act as four passes over HBM.

Backward is composed of differentiable primitives (bias_act grad op, HIP conv / transposed conv /
weight-gradient Functions, small torch reductions), so second-order passes (path-length
regulariser) differentiate through it.  The conv result c is kept from the forward for the first
order; under create_graph it is recomputed as a differentiable conv so d(dL/dd)/dW, /ds, /dx exist.
"""
import torch

from . import bias_act as _ba
from . import conv2d_gradfix as _cg

_CL = torch.channels_last
enabled = True   # switch for A/B tests against the composed (unfused) path


def supported(x, weight, up):
    n, cin, h, w = x.shape
    cout, _, kh, kw = weight.shape
    return (enabled and up == 1 and kh == 3 and kw == 3 and x.dtype in (torch.float16, torch.bfloat16) and x.is_cuda and
            cin % 8 == 0 and cout % 8 == 0 and h >= 16 and w >= 16)


class ModConvLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, styles, weight, dcoefs, noise, bias, alpha, gain, clamp):
        x = _cg._nhwc(x)
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        wT = weight.to(x.dtype)
        nz = None
        if noise is not None:
            nz = noise.to(x.dtype).reshape(n, h, w).contiguous()
        want_raw = any(ctx.needs_input_grad[:6])
        want_raw = want_raw and dcoefs is not None     # c only feeds dL/dd
        y, c = _cg.conv3x3_fused(x, _cg._pack_conv(wT), cout, in_scale=_f32(styles), out_scale=_f32(dcoefs),
                                 noise=nz, noise_gain=1.0, bias=_f32(bias), act=1, alpha=alpha, gain=gain,
                                 clamp=clamp, want_raw=want_raw)
        ctx.save_for_backward(x, styles, weight, dcoefs, noise, bias, y, c)
        ctx.cfg = (alpha, gain, clamp)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, styles, weight, dcoefs, noise, bias, y, c = ctx.saved_tensors
        alpha, gain, clamp = ctx.cfg
        n, cin, h, w = x.shape
        dt = x.dtype
        need = ctx.needs_input_grad
        if not torch.is_grad_enabled() and fast_backward:
            return _fast_backward(ctx, dy, x, styles, weight, dcoefs, noise, bias, y, c, alpha, gain, clamp)
        dz = _ba.bias_act_grad(dy, y, act='lrelu', alpha=alpha, gain=gain, clamp=clamp)
        dx = ds = dw = dd = dnoise = db = None
        if need[5] and bias is not None:
            db = dz.sum([0, 2, 3], dtype=torch.float32).to(bias.dtype)
        if need[4] and noise is not None:
            dnoise = dz.sum(1, keepdim=True, dtype=torch.float32).to(noise.dtype)
        s_ = styles.to(dt).reshape(n, -1, 1, 1) if styles is not None else None
        if need[3] and dcoefs is not None:
            if torch.is_grad_enabled():
                c_ = _cg._Conv2d.apply(_mul(x, s_), weight.to(dt), 1, (1, 1), (h, w))
            else:
                c_ = c
            dd = (dz * c_).sum([2, 3], dtype=torch.float32).to(dcoefs.dtype)
        dc = dz * dcoefs.to(dt).reshape(n, -1, 1, 1) if dcoefs is not None else dz
        if need[0] or need[1]:
            dxs = _cg._ConvT2d.apply(dc, weight.to(dt), 1, (1, 1), (h, w))
            if need[0]:
                dx = _mul(dxs, s_)
            if need[1] and styles is not None:
                ds = (dxs * x).sum([2, 3], dtype=torch.float32).to(styles.dtype)
        if need[2] and not _cg.weight_gradients_disabled:
            dw = _cg._WGrad.apply(dc, _mul(x, s_), (3, 3), 1, (1, 1)).to(weight.dtype)
        return dx, ds, dw, dd, dnoise, db, None, None, None


def _fast_backward(ctx, dy, x, styles, weight, dcoefs, noise, bias, y, c, alpha, gain, clamp):
    """First-order backward in three kernels (no create_graph):
      sg2_layer_bwd  : dz, dc = dz*d, db, dd = sum dz*c, dnoise         (one pass over dy, y, c)
      sg2_conv3x3    : dx = convT(dc, W) * s, ds = sum convT(dc, W) * x  (dgrad with scale + dot epilogue)
      sg2_conv2d_wgrad: dw = sum dc (x) (x * s)                          (modulation applied to the B operand)
    """
    need = ctx.needs_input_grad
    n, cin, h, w = x.shape
    dt = x.dtype
    d32 = dcoefs.float().contiguous() if dcoefs is not None else None
    dc, db, dd, dn = _cg.layer_bwd(dy.to(dt), y, c if (need[3] and d32 is not None) else None, d32, act=1,
                                   alpha=alpha, gain=gain, clamp=clamp, want_db=need[5] and bias is not None,
                                   want_dd=need[3] and d32 is not None, want_dnoise=need[4] and noise is not None)
    dx = ds = dw = None
    s32 = _f32(styles)
    want_ds = need[1] and styles is not None
    if need[0] or want_ds:
        wT = _cg._pack_convT(weight.to(dt).flip([2, 3]))
        if want_ds:
            dx, _, ds = _cg.conv3x3_fused(dc, wT, cin, out_scale=s32, dot_src=x)
            ds = ds.to(styles.dtype)
        else:
            dx, _ = _cg.conv3x3_fused(dc, wT, cin, out_scale=s32)
        dx = dx if need[0] else None
    if need[2] and not _cg.weight_gradients_disabled:
        dw = _cg._wgrad_raw(dc, x, 3, 3, 1, (1, 1), x_scale=s32).to(weight.dtype)
    db = db.to(bias.dtype) if db is not None else None
    dd = dd.to(dcoefs.dtype) if dd is not None else None
    dn = dn.to(noise.dtype) if dn is not None else None
    return dx, ds, dw, dd, dn, db, None, None, None


fast_backward = True   # first-order backward through the fused kernels (A/B switch)


def _f32(t):
    return t.float().contiguous() if t is not None else None


def _mul(a, s):
    return a * s if s is not None else a


def modconv_layer(x, styles, weight, dcoefs, noise, bias, alpha, gain, clamp):
    """styles / dcoefs / noise / bias may be None: with styles = dcoefs = noise = None this is the
    discriminator's plain 3x3 Conv2dLayer + bias + lrelu (networks_stylegan2.py:172-181) in one kernel."""
    return ModConvLayer.apply(x, styles, weight, dcoefs, noise, bias, float(alpha), float(gain),
                              float(clamp if clamp is not None else -1.0))
