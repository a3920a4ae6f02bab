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
        y, c = _cg.conv3x3_fused(x, _cg._pack_conv(wT), cout, in_scale=styles.float().contiguous(),
                                 out_scale=dcoefs.float().contiguous() if dcoefs is not None else None,
                                 noise=nz, noise_gain=1.0, bias=bias.float().contiguous(), act=1, alpha=alpha,
                                 gain=gain, clamp=clamp, want_raw=want_raw)
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
        dz = _ba.bias_act_grad(dy, y, act='lrelu', alpha=alpha, gain=gain, clamp=clamp)
        dx = ds = dw = dd = dnoise = db = None
        if need[5]:
            db = dz.sum([0, 2, 3], dtype=torch.float32).to(bias.dtype)
        if need[4] and noise is not None:
            dnoise = dz.sum(1, keepdim=True, dtype=torch.float32).to(noise.dtype)
        s_ = styles.to(dt).reshape(n, -1, 1, 1)
        if need[3] and dcoefs is not None:
            if torch.is_grad_enabled():
                c_ = _cg._Conv2d.apply(x * s_, weight.to(dt), 1, (1, 1), (h, w))
            else:
                c_ = c
            dd = (dz * c_).sum([2, 3], dtype=torch.float32).to(dcoefs.dtype)
        dc = dz * dcoefs.to(dt).reshape(n, -1, 1, 1) if dcoefs is not None else dz
        if need[0] or need[1]:
            dxs = _cg._ConvT2d.apply(dc, weight.to(dt), 1, (1, 1), (h, w))
            if need[0]:
                dx = dxs * s_
            if need[1]:
                ds = (dxs * x).sum([2, 3], dtype=torch.float32).to(styles.dtype)
        if need[2] and not _cg.weight_gradients_disabled:
            dw = _cg._WGrad.apply(dc, x * s_, (3, 3), 1, (1, 1)).to(weight.dtype)
        return dx, ds, dw, dd, dnoise, db, None, None, None


def modconv_layer(x, styles, weight, dcoefs, noise, bias, alpha, gain, clamp):
    return ModConvLayer.apply(x, styles, weight, dcoefs, noise, bias, float(alpha), float(gain),
                              float(clamp if clamp is not None else -1.0))
