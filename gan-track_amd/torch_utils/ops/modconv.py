"""Fused StyleGAN2 conv layers: convolution + modulation + demodulation + noise + bias + activation
(+ resnet residual) in one kernel launch, with a fused first-order backward.

Forward (reference SG3/training/networks_stylegan2.py: SynthesisLayer :309-328 with
modulated_conv2d :32-77 in its non-fused training form; Conv2dLayer :172-181; the resnet add of
DiscriminatorBlock :621-627):
    c = conv(x * s[n, ci], W)                      (modulation applied while staging x)
    z = clamp(act(c * d[n, co] + noise + b) * gain, +-clamp)
    y = z + residual                               (optional)
where the reference runs x*s, conv, fma(x, d, noise), bias_act and add as separate HBM passes.
The 3x3 / stride-1 16-bit layers run on the LDS-halo kernel (sg2_conv3x3), the 3x3 / stride-2 / pad-0
ones from 65^2 inputs on its stride-2 form (sg2_conv3x3_s2, with the resnet residual in its epilogue);
every other geometry and f32 runs on the implicit-GEMM kernel with the same epilogue (sg2_conv2d_fused).

Backward:
  * first order (no create_graph): sg2_layer_bwd (dz, dc = dz*d, db, dd, dnoise in one pass), then
    the data gradient with the `*s` scale (and on the halo kernel the `ds` dot reduction) in its
    epilogue, and the weight gradient with the modulation applied to its B operand;
  * under create_graph (path-length / R1 double backward) the same gradient is composed of
    differentiable primitives (bias_act grad op, HIP conv / transposed conv / weight-gradient
    Functions), and c is recomputed as a differentiable conv so d(dL/dd)/dW, /ds, /dx exist.
"""
import os

import torch

from . import bias_act as _ba
from . import conv2d_gradfix as _cg
from . import staged_sum as _ss
from . import upfirdn2d as _up

_CL = torch.channels_last
enabled = True         # switch for A/B tests against the composed (unfused) path
prezero = os.environ.get('SG2_PREZERO', '1') != '0'   # one zero fill per layer backward (A/B switch)
# deterministic mode: the library's slot sums assign the accumulators instead of adding into zeros, so the layer
# backward allocates them unfilled (SG2_DET_ASSIGN=0: the former fill + add; the library reads the same switch)
det_assign = os.environ.get('SG2_DET_ASSIGN', '1') != '0'
fast_backward = True   # first-order backward through the fused kernels (A/B switch)
fused_vjp = os.environ.get('SG2_FUSED_VJP', '1') != '0'   # create_graph input-gradient pass as one node (A/B)
tap_enabled = os.environ.get('SG2_TORGB_TAP', '1') != '0'   # toRGB input gradient + next block's in one epilogue
_ACT = {0: 'linear', 1: 'lrelu'}


def supported(x, weight, up):
    """The 3x3 up=1 synthesis / D layer on the LDS-halo kernel (16-bit, >= 16^2)."""
    n, cin, h, w = x.shape
    cout, _, kh, kw = weight.shape
    return (enabled and up == 1 and kh == 3 and kw == 3 and x.dtype in (torch.float16, torch.bfloat16) and x.is_cuda and
            cin % 8 == 0 and cout % 8 == 0 and h >= 16 and w >= 16)


def supported_generic(x, weight):
    """Any other geometry / dtype on the implicit-GEMM kernel."""
    return enabled and x.is_cuda


def _halo(x, kh, kw, stride, pad):
    n, cin, h, w = x.shape
    return (kh == 3 and kw == 3 and stride == 1 and pad == 1 and x.dtype in (torch.float16, torch.bfloat16) and
            cin % 8 == 0 and h >= 16 and w >= 16)


def _f32(t):
    return t.float().contiguous() if t is not None else None


def _sum_hw(t):
    """t.sum([2, 3], dtype=float32) as [N, C] without torch's split reduction (staged_sum.py)."""
    return _ss.staged_sum(t, (2, 3), dtype=torch.float32)


def _sum_nhw(t):
    """t.sum([0, 2, 3], dtype=float32) (a bias gradient) without torch's split reduction (staged_sum.py)."""
    return _ss.staged_sum(t, (0, 2, 3), dtype=torch.float32)


def _mul(a, s):
    return a * s if s is not None else a


class FusedConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, styles, weight, dcoefs, noise, bias, residual, stride, pad, act, alpha, gain, clamp, wgain):
        # wgain: the layer's weight gain (Conv2dLayer's `weight * weight_gain`, networks_stylegan2.py:173), applied
        # by the weight pack and by the weight-gradient kernel instead of two elementwise launches
        x_in = x                       # saved as given: a create_graph backward differentiates through it
        x = _cg._nhwc(x)
        n, cin, h, w = x.shape
        cout, _, kh, kw = weight.shape
        oh = (h + 2 * pad - kh) // stride + 1
        ow = (w + 2 * pad - kw) // stride + 1
        dt = x.dtype
        nz = noise.to(dt).reshape(n, oh, ow).contiguous() if noise is not None else None
        any_grad = any(ctx.needs_input_grad[:7])
        want_c = any_grad and dcoefs is not None          # c feeds dL/dd
        want_z = any_grad and residual is not None        # z = y - residual feeds the activation grad
        assert not (want_c and want_z), 'demodulation and a residual in one layer are not supported'
        b32 = _f32(bias) if bias is not None else None   # the kernels add it rounded to x.dtype, as the reference
        if _halo(x, kh, kw, stride, pad) and residual is None:
            y, aux = _cg.conv3x3_fused(x, _cg._pack_conv(weight, dt, scale=wgain), cout, in_scale=_f32(styles), out_scale=_f32(dcoefs),
                                       noise=nz, noise_gain=1.0, bias=b32, act=act, alpha=alpha, gain=gain,
                                       clamp=clamp, want_raw=want_c)
        elif _cg._halo_s2_ok(x, kh, kw, stride, pad, cout=cout, scaled=styles is not None or noise is not None):
            y, aux = _cg.conv3x3_fused(x, _cg._pack_conv(weight, dt, scale=wgain), cout, in_scale=_f32(styles),
                                       out_scale=_f32(dcoefs), noise=nz, noise_gain=1.0, bias=b32, act=act,
                                       alpha=alpha, gain=gain, clamp=clamp, want_raw=want_c or want_z, stride=2,
                                       residual=residual, raw_act=want_z)
        else:
            y, aux = _cg.conv_fused(x, _cg._pack_conv(weight, dt, scale=wgain), cout, oh, ow, kh, kw, stride, (pad, pad),
                                    in_scale=_f32(styles), out_scale=_f32(dcoefs), noise=nz, noise_gain=1.0,
                                    bias=b32, act=act, alpha=alpha, gain=gain, clamp=clamp, residual=residual,
                                    aux_mode=1 if want_c else (2 if want_z else 0))
        ctx.save_for_backward(x_in, styles, weight, dcoefs, noise, bias, y, aux)
        ctx.cfg = (stride, pad, act, alpha, gain, clamp, residual is not None, wgain)
        return y

    @staticmethod
    def backward(ctx, dy):
        need = ctx.needs_input_grad
        g = _fused_conv_grads(ctx, need, dy)
        return g + (dy if need[6] else None, None, None, None, None, None, None, None)


def _fused_conv_grads(ctx, need, dy, dx_residual=None):
    """(dx, ds, dw, dd, dnoise, db) of a FusedConv node.  dx_residual: a gradient to add to dx (FusedConvTap: the
    other consumer's gradient of the layer input), inside the dgrad epilogue on the first-order fast path."""
    x, styles, weight, dcoefs, noise, bias, y, aux = ctx.saved_tensors
    stride, pad, act, alpha, gain, clamp, has_res, wgain = ctx.cfg
    zsrc = aux if has_res else y
    c = aux if (dcoefs is not None and not has_res) else None
    if not torch.is_grad_enabled() and fast_backward:
        return _fast_backward(need, dy, _cg._nhwc(x), styles, weight, dcoefs, noise, bias, zsrc, c, stride, pad, act,
                              alpha, gain, clamp, wgain, dx_residual=dx_residual)
    if fused_vjp and _cg.weight_gradients_disabled and not has_res and (dcoefs is None or c is not None):
        # the path-length / R1 pass: input gradients only, as one node with fused kernels both ways
        dx, ds, dd = _LayerVJP.apply(dy, x, styles, weight, dcoefs, zsrc, c, need[0], need[1], need[3],
                                     stride, pad, act, alpha, gain, clamp, wgain)
        g = (dx, ds, None, dd, None, None)
    else:
        g = _composed_backward(need, dy, x, styles, weight, dcoefs, noise, bias, zsrc, c, stride, pad, act, alpha,
                               gain, clamp, wgain)
    if dx_residual is not None and g[0] is not None:
        # in the input's dtype first, as autograd rounds each gradient before it sums them
        g = (g[0].to(dx_residual.dtype) + dx_residual,) + tuple(g[1:])
    return g


class FusedConvTap(torch.autograd.Function):
    """FusedConv (a toRGB layer: no demodulation, noise or residual) that also passes its input through as a second
    output -- the synthesis block's feature map, which feeds both the toRGB layer and the next block
    (networks_stylegan2.py SynthesisBlock.forward; reference :446-455).  Autograd would add the two consumers'
    gradients of the map in an activation-sized pass; this node receives both and, on the first-order fast path, adds
    the pass-through gradient inside the toRGB input gradient's epilogue (the conv epilogue's residual: round(dx) +
    g, the sum autograd forms)."""

    @staticmethod
    def forward(ctx, x, styles, weight, bias, pad, clamp):
        y = FusedConv.forward(ctx, x, styles, weight, None, None, bias, None, 1, pad, 0, 0.2, 1.0, clamp, 1.0)
        return x.view_as(x), y

    @staticmethod
    def backward(ctx, g_pass, dy):
        n = ctx.needs_input_grad
        need = (n[0], n[1], n[2], False, False, n[3], False)
        if dy is None:
            return g_pass, None, None, None, None, None
        res = None
        if g_pass is not None and n[0]:
            res = _cg._nhwc(g_pass.to(ctx.saved_tensors[0].dtype))
        dx, ds, dw, _, _, db = _fused_conv_grads(ctx, need, dy, dx_residual=res)
        if dx is None and res is not None:
            dx = res
        return dx, ds, dw, db, None, None


def fused_conv_tap(x, weight, styles, bias, padding, clamp):
    """(x, fused_conv(x, weight, styles=styles, bias=bias, padding=padding, clamp=clamp)) through FusedConvTap."""
    return FusedConvTap.apply(x, styles, weight, bias, int(padding), float(clamp if clamp is not None else -1.0))


def _scaled_input_grads(dc, x, styles, weight, need_x, need_s, need_w, stride, pad, wgain=1.0, acc_ds=None,
                        acc_dw=None, dx_residual=None):
    """Gradients of c = conv(x * s, W) given dc: dx = convT(dc, W) * s and ds = sum_hw convT(dc, W) * x in
    one dgrad launch (out_scale / dot_src epilogue), dw = the s-scaled weight gradient.  acc_ds / acc_dw:
    zeroed f32 buffers (N*Cin / Cout*kh*kw*Cin) the reductions accumulate into (no memset per call).
    dx_residual: added to dx in the epilogue (round(dx) + residual; FusedConvTap)."""
    n, cin, h, w = x.shape
    cout, _, kh, kw = weight.shape
    dt = x.dtype
    dx = ds = dw = None
    s32 = _f32(styles)
    want_ds = need_s and styles is not None
    dso = acc_ds.view(n, cin) if (want_ds and acc_ds is not None) else None
    if need_x or want_ds:
        if dx_residual is not None and not need_x:
            dx_residual = None
        if _halo(dc, kh, kw, stride, pad) and dx_residual is None:
            wT = _cg._pack_convT(weight, dt, flip=True, scale=wgain)
            if want_ds:
                dx, _, ds = _cg.conv3x3_fused(dc, wT, cin, out_scale=s32, dot_src=x, dot_out=dso)
            else:
                dx, _ = _cg.conv3x3_fused(dc, wT, cin, out_scale=s32)
        else:
            if want_ds:
                dx, _, ds = _cg.conv_fused(dc, _cg._pack_convT(weight, dt, scale=wgain), cin, h, w, kh, kw, stride,
                                           (pad, pad), transpose=True, out_scale=s32, dot_src=x, dot_out=dso,
                                           residual=dx_residual)
            else:
                dx, _ = _cg.conv_fused(dc, _cg._pack_convT(weight, dt, scale=wgain), cin, h, w, kh, kw, stride,
                                       (pad, pad), transpose=True, out_scale=s32, residual=dx_residual)
        ds = ds.to(styles.dtype) if want_ds else None
        dx = dx if need_x else None
    if need_w and not _cg.weight_gradients_disabled:
        dw = _cg._wgrad_raw(dc, x, kh, kw, stride, (pad, pad), x_scale=s32, alpha=wgain, out=acc_dw,
                            param_layout=True).to(weight.dtype)
    return dx, ds, dw


class _ScaledConvT(torch.autograd.Function):
    """dxs = convT(dz * d, W), the create_graph backward's dgrad with the demodulation scale d [N, Cout] on
    the operand staging (no dz * d pass in HBM).  Backward: one conv launch gives d(dz) = conv(G, W) * d
    (out_scale) and dd = sum_p conv(G, W) * dz (dot_src); dW is the d-scaled weight gradient.  A third
    order falls back to differentiating the composed form."""

    @staticmethod
    def forward(ctx, dz, d, weight, stride, pad, out_hw):
        dzk = _cg._nhwc(dz)            # the kernels' layout; the input itself is saved (third-order fallback)
        cin, kh, kw = weight.shape[1], weight.shape[2], weight.shape[3]
        dt = dz.dtype
        if _halo(dzk, kh, kw, stride, pad):
            y, _ = _cg.conv3x3_fused(dzk, _cg._pack_convT(weight, dt, flip=True), cin, in_scale=_f32(d))
        else:
            y, _ = _cg.conv_fused(dzk, _cg._pack_convT(weight, dt), cin, out_hw[0], out_hw[1], kh, kw, stride,
                                  (pad, pad), transpose=True, in_scale=_f32(d))
        ctx.save_for_backward(dz, d, weight)
        ctx.cfg = (stride, pad, tuple(out_hw))
        return y

    @staticmethod
    def backward(ctx, g):
        dz, d, weight = ctx.saved_tensors
        stride, pad, out_hw = ctx.cfg
        need = ctx.needs_input_grad
        dt = dz.dtype
        n, cout, oh, ow = dz.shape
        kh, kw = weight.shape[2], weight.shape[3]
        if torch.is_grad_enabled():
            ins = [t for t, nd in zip((dz, d, weight), need[:3]) if nd]
            y = _cg._ConvT2d.apply(dz * d.to(dt).reshape(n, -1, 1, 1), weight.to(dt), stride, (pad, pad), out_hw)
            gs = iter(torch.autograd.grad(y, ins, g, create_graph=True, allow_unused=True))
            return tuple(next(gs) if nd else None for nd in need[:3]) + (None, None, None)
        g = _cg._nhwc(g.to(dt))
        dz = _cg._nhwc(dz)
        d32 = _f32(d)
        gdz = gd = gw = None
        if need[0] or need[1]:
            src = dz if need[1] else None
            if _halo(g, kh, kw, stride, pad):
                res = _cg.conv3x3_fused(g, _cg._pack_conv(weight, dt), cout, out_scale=d32, dot_src=src)
            else:
                res = _cg.conv_fused(g, _cg._pack_conv(weight, dt), cout, oh, ow, kh, kw, stride, (pad, pad),
                                     out_scale=d32, dot_src=src)
            gdz = res[0] if need[0] else None
            gd = res[2].to(d.dtype) if need[1] else None
        if need[2] and not _cg.weight_gradients_disabled:
            gw = _cg._wgrad_raw(dz, g, kh, kw, stride, (pad, pad), g_scale=d32).to(weight.dtype)
        return gdz, gd, gw, None, None, None


class _SavedRaw(torch.autograd.Function):
    """c = conv(x * s, W), the layer's raw (pre-demodulation) conv output, as a differentiable value for the
    create_graph backward (dL/dd = sum_hw dz * c).  The forward hands back the c the fused forward kernel
    already wrote (aux) instead of recomputing the modulated conv; the backward is the first-order
    _scaled_input_grads (the reference differentiates the recomputed grouped conv, networks_stylegan2.py:80-89).
    A third order falls back to differentiating a recomputed conv."""

    @staticmethod
    def forward(ctx, x, styles, weight, c, stride, pad):
        ctx.save_for_backward(x, styles, weight)
        ctx.cfg = (stride, pad)
        return c.view_as(c)

    @staticmethod
    def backward(ctx, dc):
        x, styles, weight = ctx.saved_tensors
        stride, pad = ctx.cfg
        need = ctx.needs_input_grad
        if torch.is_grad_enabled():
            dt = x.dtype
            n = x.shape[0]
            oh, ow = dc.shape[2], dc.shape[3]
            ins = [t for t, nd in zip((x, styles, weight), need[:3]) if nd]
            cc = _cg._Conv2d.apply(_mul(x, styles.to(dt).reshape(n, -1, 1, 1)), weight.to(dt), stride, (pad, pad),
                                   (oh, ow))
            gs = iter(torch.autograd.grad(cc, ins, dc, create_graph=True, allow_unused=True))
            return tuple(next(gs) if nd else None for nd in need[:3]) + (None, None, None)
        dx, ds, dw = _scaled_input_grads(_cg._nhwc(dc.to(x.dtype)), _cg._nhwc(x), styles,
                                         weight, need[0], need[1], need[2], stride, pad)
        return dx, ds, dw, None, None, None


def _conv_any(x, weight, cout, oh, ow, stride, pad, transpose, wgain, **epi):
    """One fused conv launch of the layer geometry: the LDS-halo kernel for 16-bit 3x3/s1/p1, the implicit GEMM
    otherwise.  transpose: the input gradient's convT (weight [Cout, Cin, kh, kw] read as its adjoint).  epi:
    in_scale / out_scale / dot_src / want_raw.  Returns (y, raw or None, dot or None)."""
    kh, kw = weight.shape[2], weight.shape[3]
    dt = x.dtype
    want_raw = epi.pop('want_raw', False)
    dot_src = epi.get('dot_src')
    if _halo(x, kh, kw, stride, pad):
        wp = _cg._pack_convT(weight, dt, flip=True, scale=wgain) if transpose else _cg._pack_conv(weight, dt, scale=wgain)
        res = _cg.conv3x3_fused(x, wp, cout, want_raw=want_raw, **epi)
    else:
        wp = _cg._pack_convT(weight, dt, scale=wgain) if transpose else _cg._pack_conv(weight, dt, scale=wgain)
        res = _cg.conv_fused(x, wp, cout, oh, ow, kh, kw, stride, (pad, pad), transpose=transpose,
                             aux_mode=1 if want_raw else 0, **epi)
    return res[0], res[1], (res[2] if dot_src is not None else None)


class _LayerVJP(torch.autograd.Function):
    """The layer's input-gradient VJP as one differentiable node: the path-length pass (loss.py pl_no_weight_grad,
    reference loss.py:85-100 under conv2d_gradfix.no_weight_gradients) and R1's create_graph pass differentiate it
    once more.  For z = act(c * d + noise + b) * gain, c = conv(x * s, W):
        forward    dc = act'(dy; y) * d, dd = sum_hw act'(dy; y) * c      (sg2_layer_bwd, one pass)
                   dxs = convT(dc, W); dx = dxs * s; ds = sum_hw dxs * x     (one dgrad launch, raw dxs kept)
        backward   G = g_dx * s + g_ds * x
                   A = conv(G, W):  g_dy = act'(A * d + g_dd * c; y),  g_d = sum_hw A * dc / d
                   H = g_dd * act'(dy; y) = dc * (g_dd / d):
                       g_x = g_ds * dxs + convT(H, W) * s,   g_s = sum_hw g_dx * dxs + sum_hw convT(H, W) * x
                   g_W = wgrad(dc, G) + wgrad(dc * g_dd / d, x * s)   (x wgain for the raw weight)
    (act' of lrelu / linear is piecewise constant in y: no second-order term in y, as the reference's bias_act grad.)
    Each conv is one fused launch with its scales on the operand staging and its reductions in the epilogue, where
    the composed form runs the conv recompute, two dot kernels and the elementwise products as separate nodes."""

    @staticmethod
    def forward(ctx, dy, x, styles, weight, dcoefs, zsrc, c, need_x, need_s, need_d, stride, pad, act, alpha, gain,
                clamp, wgain):
        xk = _cg._nhwc(x)
        n, cin, h, w = xk.shape
        cout = weight.shape[0]
        dt = xk.dtype
        d32, s32 = _f32(dcoefs), _f32(styles)
        want_dd = need_d and d32 is not None
        want_ds = need_s and s32 is not None
        if zsrc.shape[1] % 8 == 0:
            dc, _, dd, _ = _cg.layer_bwd(dy.to(dt), zsrc, c if want_dd else None, d32, act=act, alpha=alpha, gain=gain,
                                         clamp=clamp, want_db=False, want_dd=want_dd, want_dnoise=False)
        else:   # narrow outputs (toRGB)
            dz = _ba.bias_act_grad(dy.to(dt), zsrc, act=_ACT[act], alpha=alpha, gain=gain, clamp=clamp)
            dd = _sum_hw(dz * c) if want_dd else None
            dc = _cg._nhwc(dz * dcoefs.to(dt).reshape(n, -1, 1, 1) if d32 is not None else dz)
        dx, dxs, ds = _conv_any(dc, weight, cin, h, w, stride, pad, True, wgain, out_scale=s32,
                                dot_src=xk if want_ds else None, want_raw=s32 is not None)
        if dxs is None:
            dxs = dx
        ctx.save_for_backward(xk, styles, weight, dcoefs, zsrc, c, dc, dxs)
        ctx.cfg = (stride, pad, act, alpha, gain, clamp, wgain)
        return (dx if need_x else None, ds.to(styles.dtype) if want_ds else None,
                dd.to(dcoefs.dtype) if want_dd else None)

    @staticmethod
    def backward(ctx, g_dx, g_ds, g_dd):
        if torch.is_grad_enabled():
            raise RuntimeError('_LayerVJP: third-order gradients are not supported (set modconv.fused_vjp = False)')
        x, styles, weight, dcoefs, zsrc, c, dc, dxs = ctx.saved_tensors
        stride, pad, act, alpha, gain, clamp, wgain = ctx.cfg
        need = ctx.needs_input_grad
        n, cin, h, w = x.shape
        cout, _, kh, kw = weight.shape
        oh, ow = dc.shape[2], dc.shape[3]
        dt = x.dtype
        d32, s32 = _f32(dcoefs), _f32(styles)
        g_dy = g_x = g_s = g_w = g_d = None
        g_ds = g_ds if s32 is not None else None
        gds32 = _f32(g_ds)
        # G = dL/d(dxs) = g_dx * s + g_ds * x, with sum_p g_dx * dxs (the direct part of g_s) in the same pass
        G = None
        if g_dx is not None and s32 is None:      # (an unmodulated layer: G is g_dx itself)
            G = _cg._nhwc(g_dx.to(dt))
        elif g_dx is not None:
            G, g_s = _cg.vjp_axpy(g_dx.to(dt), s32, x if g_ds is not None else None, gds32,
                                  e=dxs if need[2] else None)
        elif g_ds is not None:
            G, _ = _cg.vjp_axpy(x, gds32)
        hscale = (g_dd.float() / d32).contiguous() if (g_dd is not None and d32 is not None) else None
        if G is not None and (need[0] or need[4]):
            A_d, _, dot = _conv_any(G, weight, cout, oh, ow, stride, pad, False, wgain, out_scale=d32,
                                    dot_src=dc if (need[4] and d32 is not None) else None)
            if need[4] and d32 is not None:
                g_d = (dot / d32).to(dcoefs.dtype)
            if need[0]:   # g_dy = act'(A d + g_dd * c; y): one pass
                g_dy, _ = _cg.vjp_axpy(A_d, None, c if hscale is not None else None, _f32(g_dd) if hscale is not None
                                       else None, y=zsrc, act=act, alpha=alpha, gain=gain, clamp=clamp)
        elif need[0] and hscale is not None:
            g_dy, _ = _cg.vjp_axpy(c, _f32(g_dd), y=zsrc, act=act, alpha=alpha, gain=gain, clamp=clamp)
        if need[1] or need[2]:
            gxc = gsc = None
            if hscale is not None:
                gxc, _, gsc = _conv_any(dc, weight, cin, h, w, stride, pad, True, wgain, in_scale=hscale,
                                        out_scale=s32, dot_src=x if (need[2] and s32 is not None) else None)
            if need[1]:   # g_x = convT(H, W) * s + g_ds * dxs: one pass
                if g_ds is not None:
                    g_x, _ = (_cg.vjp_axpy(gxc, None, dxs, gds32) if gxc is not None else _cg.vjp_axpy(dxs, gds32))
                else:
                    g_x = gxc
            if gsc is not None:
                g_s = gsc if g_s is None else g_s + gsc
        if need[3] and (G is not None or hscale is not None):
            acc = torch.zeros([cout * kh * kw * cin], dtype=torch.float32, device=x.device)
            # (both calls take the same kernel path, so they agree on acc's layout; the returned view reads it)
            if G is not None:
                g_w = _cg._wgrad_raw(dc, G, kh, kw, stride, (pad, pad), alpha=wgain, out=acc, param_layout=True)
            if hscale is not None:
                g_w = _cg._wgrad_raw(dc, x, kh, kw, stride, (pad, pad), x_scale=s32, g_scale=hscale, alpha=wgain,
                                     out=acc, param_layout=True)
            g_w = g_w.to(weight.dtype)
        g_s = g_s.to(styles.dtype) if g_s is not None else None
        return (g_dy, g_x, g_s, g_w, g_d) + (None,) * 12


def _fast_backward(need, dy, x, styles, weight, dcoefs, noise, bias, zsrc, c, stride, pad, act, alpha, gain, clamp,
                   wgain=1.0, dx_residual=None):
    """First order in three kernels: sg2_layer_bwd; dgrad with the *s scale (+ ds); scaled wgrad."""
    n, cin, h, w = x.shape
    cout, _, kh, kw = weight.shape
    dt = x.dtype
    d32 = _f32(dcoefs)
    want_dd = need[3] and d32 is not None
    want_db, want_dn = need[5] and bias is not None, need[4] and noise is not None
    # one zero fill for all of the layer's float accumulators (db, dd, ds, dw) instead of a memset per kernel
    wide = zsrc.shape[1] % 8 == 0
    want_ds = need[1] and styles is not None and (need[0] or need[1])
    want_dw = need[2] and not _cg.weight_gradients_disabled
    sizes = [cout if (wide and want_db) else 0, n * cout if (wide and want_dd) else 0, n * cin if want_ds else 0,
             cout * kh * kw * cin if want_dw else 0]
    if not prezero or (det_assign and _cg._hip.det_active()):   # deterministic: each slot sum assigns (no fill)
        sizes = [0, 0, 0, 0]
    acc = torch.zeros([sum(sizes)], dtype=torch.float32, device=dy.device) if sum(sizes) else None
    parts, o = [], 0
    for k in sizes:
        parts.append(acc[o:o + k] if k else None)
        o += k
    if wide:
        lb = acc[:sizes[0] + sizes[1]] if sizes[0] + sizes[1] else None
        dc, db, dd, dn = _cg.layer_bwd(dy.to(dt), zsrc, c if want_dd else None, d32, act=act, alpha=alpha, gain=gain,
                                       clamp=clamp, want_db=want_db, want_dd=want_dd, want_dnoise=want_dn, acc=lb)
    else:   # narrow outputs (toRGB): plain kernels
        dz = _ba.bias_act_grad(dy, zsrc, act=_ACT[act], alpha=alpha, gain=gain, clamp=clamp)
        db = _sum_nhw(dz) if want_db else None
        dd = _sum_hw(dz * c) if want_dd else None
        dn = dz.sum(1, keepdim=True, dtype=torch.float32) if want_dn else None
        dc = _cg._nhwc(dz * dcoefs.to(dt).reshape(n, -1, 1, 1) if dcoefs is not None else dz)
    dx, ds, dw = _scaled_input_grads(dc, x, styles, weight, need[0], need[1], need[2], stride, pad, wgain,
                                     acc_ds=parts[2], acc_dw=parts[3], dx_residual=dx_residual)
    db = db.to(bias.dtype) if db is not None else None
    dd = dd.to(dcoefs.dtype) if dd is not None else None
    dn = dn.to(noise.dtype) if dn is not None else None
    return dx, ds, dw, dd, dn, db


def _composed_backward(need, dy, x, styles, weight, dcoefs, noise, bias, zsrc, c, stride, pad, act, alpha, gain,
                       clamp, wgain=1.0):
    """Differentiable form (used under create_graph).  With a weight gain the convolutions see weight * wgain
    (a differentiable op, so the second-order terms reach the raw weight), and the weight gradient is
    returned for the RAW weight: dL/dW = wgain * dL/d(W * wgain)."""
    if wgain != 1.0:
        weight = weight * wgain        # (rare path: the R1 double backward) the gain as a differentiable op
    n, cin, h, w = x.shape
    cout, _, kh, kw = weight.shape
    oh, ow = zsrc.shape[2], zsrc.shape[3]
    dt = x.dtype
    dz = _ba.bias_act_grad(dy, zsrc, act=_ACT[act], alpha=alpha, gain=gain, clamp=clamp)
    dx = ds = dw = dd = dnoise = db = None
    # Under no_weight_gradients() (the path-length pass, loss.py pl_no_weight_grad) the caller asks for
    # input gradients only (autograd.grad(..., inputs=[ws])): the parameter gradients db / dnoise would
    # be computed and discarded, and -- being differentiable -- add their own double-backward nodes.
    param_grads = not _cg.weight_gradients_disabled
    if need[5] and bias is not None and param_grads:
        db = _sum_nhw(dz).to(bias.dtype)
    if need[4] and noise is not None and param_grads:
        dnoise = dz.sum(1, keepdim=True, dtype=torch.float32).to(noise.dtype)
    s_ = styles.to(dt).reshape(n, -1, 1, 1) if styles is not None else None
    if need[3] and dcoefs is not None:
        if torch.is_grad_enabled() and c is not None and styles is not None:
            c_ = _SavedRaw.apply(x, styles, weight, c, stride, pad)
        elif torch.is_grad_enabled():
            c_ = _cg._Conv2d.apply(_mul(x, s_), weight.to(dt), stride, (pad, pad), (oh, ow))
        else:
            c_ = c
        dd = _cg.dot_hw(dz, c_).to(dcoefs.dtype)
    want_dw = need[2] and not _cg.weight_gradients_disabled
    scaled_t = dcoefs is not None and not want_dw       # the PL pass: dc feeds the dgrad only
    dc = dz * dcoefs.to(dt).reshape(n, -1, 1, 1) if dcoefs is not None and not scaled_t else dz
    if need[0] or need[1]:
        if scaled_t:
            dxs = _ScaledConvT.apply(dz, dcoefs, weight, stride, pad, (h, w))
        else:
            dxs = _cg._ConvT2d.apply(dc, weight.to(dt), stride, (pad, pad), (h, w))
        if need[0]:
            dx = _mul(dxs, s_)
        if need[1] and styles is not None:
            ds = _cg.dot_hw(dxs, x).to(styles.dtype)
    if need[2] and not _cg.weight_gradients_disabled:
        dw = _cg._WGrad.apply(dc, _mul(x, s_), (kh, kw), stride, (pad, pad))
        dw = (dw * wgain if wgain != 1.0 else dw).to(weight.dtype)
    return dx, ds, dw, dd, dnoise, db


def fused_conv(x, weight, styles=None, dcoefs=None, noise=None, bias=None, residual=None, stride=1, padding=0,
               act='linear', alpha=0.2, gain=1.0, clamp=None, wgain=1.0):
    """wgain: multiplier of `weight` (a Conv2dLayer's weight gain), applied inside the weight pack and the
    weight-gradient kernel."""
    return FusedConv.apply(x, styles, weight, dcoefs, noise, bias, residual, int(stride), int(padding),
                           1 if act == 'lrelu' else 0, float(alpha), float(gain),
                           float(clamp if clamp is not None else -1.0), float(wgain))


def modconv_layer(x, styles, weight, dcoefs, noise, bias, alpha, gain, clamp):
    """3x3 modulated synthesis layer (lrelu).  With styles = dcoefs = noise = None this is the
    discriminator's plain 3x3 Conv2dLayer + bias + lrelu (networks_stylegan2.py:172-181)."""
    return fused_conv(x, weight, styles=styles, dcoefs=dcoefs, noise=noise, bias=bias, padding=1, act='lrelu',
                      alpha=alpha, gain=gain, clamp=clamp)


# ---------------------------------------------------------------------------------------------- up-2
def _up_geometry(h, w, kh, kw, f):
    """Padding algebra of conv2d_resample's transposed plan (conv2d_resample.py:112-129) for a
    padding-1 / up-2 layer: transposed-conv padding, its output size and the FIR padding."""
    from . import conv2d_resample as _cr
    x0, x1, y0, y1 = _cr._frame_padding(kw // 2, f, 2, 1)
    x0, x1 = x0 - (kw - 1), x1 - (kw - 2)
    y0, y1 = y0 - (kh - 1), y1 - (kh - 2)
    cx = max(-max(x0, x1), 0)
    cy = max(-max(y0, y1), 0)
    th, tw = (h - 1) * 2 - 2 * cy + kh, (w - 1) * 2 - 2 * cx + kw
    return (cy, cx), (th, tw), [x0 + cx, x1 + cx, y0 + cy, y1 + cy]


def supported_up(x, weight, f):
    n, cin, h, w = x.shape
    cout = weight.shape[0]
    vec = 8 if x.dtype != torch.float32 else 4
    return enabled and x.is_cuda and f is not None and f.ndim == 2 and cout % vec == 0 and cout % 8 == 0


class UpModConv(torch.autograd.Function):
    """Up-2 synthesis layer (networks_stylegan2.py:309-328; modulated_conv2d :66-76 with
    conv2d_resample's transposed plan :112-129):
        t = conv_transpose2d(x * s, W^T, stride 2)     modulation folded into the conv's operand staging
        c = FIR(t) * 4                                 4x4 [1,3,3,1] filter
        y = clamp(lrelu(c * d + noise + b) * gain)     epilogue of the FIR kernel
    Two launches where the reference runs x*s, conv_transpose2d, upfirdn2d, fma and bias_act."""

    @staticmethod
    def forward(ctx, x, styles, weight, dcoefs, noise, bias, f, alpha, gain, clamp):
        x = _cg._nhwc(x)
        n, cin, h, w = x.shape
        cout, _, kh, kw = weight.shape
        dt = x.dtype
        tpad, (th, tw), fpad = _up_geometry(h, w, kh, kw, f)
        t, _ = _cg.conv_fused(x, _cg._pack_conv(weight, dt), cout, th, tw, kh, kw, 2, tpad, transpose=True,
                              in_scale=_f32(styles))
        oh, ow = th + fpad[2] + fpad[3] - f.shape[0] + 1, tw + fpad[0] + fpad[1] - f.shape[1] + 1
        nz = noise.to(dt).reshape(n, oh, ow).contiguous() if noise is not None else None
        want_c = any(ctx.needs_input_grad[:6]) and dcoefs is not None
        b32 = _f32(bias) if bias is not None else None       # rounded to x.dtype in the kernel
        y, c = _up.fir_fused(t, f, fpad, gain=4.0, out_scale=_f32(dcoefs), noise=nz, bias=b32, act=1, alpha=alpha,
                             act_gain=gain, clamp=clamp, aux_mode=1 if want_c else 0)
        ctx.save_for_backward(x, styles, weight, dcoefs, noise, bias, f, y, c)
        ctx.cfg = (alpha, gain, clamp, tpad, (th, tw), fpad)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, styles, weight, dcoefs, noise, bias, f, y, c = ctx.saved_tensors
        alpha, gain, clamp, tpad, (th, tw), fpad = ctx.cfg
        need = ctx.needs_input_grad
        n, cin, h, w = x.shape
        cout, _, kh, kw = weight.shape
        dt = x.dtype
        oh, ow = y.shape[2], y.shape[3]
        aup, adown, apad, aflip = _up.adjoint_params(f, (th, tw), (oh, ow), 1, 1, fpad, False)
        dx = ds = dw = dd = dn = db = None
        if torch.is_grad_enabled() and fused_vjp and _cg.weight_gradients_disabled and c is not None:
            # the path-length pass: input gradients only, one node with fused kernels both ways
            dx, ds, dd = _UpLayerVJP.apply(dy, x, styles, weight, dcoefs, y, c, f, need[0], need[1], need[3],
                                           alpha, gain, clamp, tpad, (th, tw), fpad)
            return (dx, ds, None, dd, None, None, None, None, None, None)
        if not torch.is_grad_enabled() and fast_backward:
            d32, s32 = _f32(dcoefs), _f32(styles)
            want_dd = need[3] and d32 is not None
            dc, db, dd, dn = _cg.layer_bwd(dy.to(dt), y, c if want_dd else None, d32, act=1, alpha=alpha, gain=gain,
                                           clamp=clamp, want_db=need[5] and bias is not None, want_dd=want_dd,
                                           want_dnoise=need[4] and noise is not None)
            dt_ = _up.upfirdn2d(dc, f, up=aup, down=adown, padding=apad, flip_filter=aflip, gain=4)
            if (need[0] or need[1]) and _cg._halo_s2_ok(dt_, kh, kw, 2, tpad, dot=need[1]):
                res = _cg.conv3x3_fused(dt_, _cg._pack_conv(weight.transpose(0, 1), dt), cin, out_scale=s32,
                                        dot_src=x if need[1] else None, stride=2)
                dx = res[0] if need[0] else None
                ds = res[2] if need[1] else None
            elif need[0] or need[1]:
                if need[1]:
                    dx, _, ds = _cg.conv_fused(dt_, _cg._pack_conv(weight.transpose(0, 1), dt), cin, h, w, kh, kw, 2, tpad, out_scale=s32,
                                               dot_src=x)
                else:
                    dx, _ = _cg.conv_fused(dt_, _cg._pack_conv(weight.transpose(0, 1), dt), cin, h, w, kh, kw, 2, tpad, out_scale=s32)
                dx = dx if need[0] else None
            if need[2] and not _cg.weight_gradients_disabled:
                dw = _cg._wgrad_raw(x, dt_, kh, kw, 2, tpad, g_scale=s32, param_layout='swap').transpose(0, 1) \
                    .to(weight.dtype)
        else:
            wt = weight.to(dt).transpose(0, 1)                # conv_transpose2d weight [Cin, Cout, kh, kw]
            dz = _ba.bias_act_grad(dy, y, act='lrelu', alpha=alpha, gain=gain, clamp=clamp)
            param_grads = not _cg.weight_gradients_disabled      # see _composed_backward
            if need[5] and bias is not None and param_grads:
                db = _sum_nhw(dz)
            if need[4] and noise is not None and param_grads:
                dn = dz.sum(1, keepdim=True, dtype=torch.float32)
            s_ = styles.to(dt).reshape(n, -1, 1, 1)
            xs = x * s_
            if need[3] and dcoefs is not None:
                t_ = _cg._ConvT2d.apply(xs, wt, 2, tpad, (th, tw))
                c_ = _up.upfirdn2d(t_, f, padding=fpad, gain=4)
                dd = _cg.dot_hw(dz, c_)
            dc = dz * dcoefs.to(dt).reshape(n, -1, 1, 1)
            dt_ = _up.upfirdn2d(dc, f, up=aup, down=adown, padding=apad, flip_filter=aflip, gain=4)
            if need[0] or need[1]:
                dxs = _cg._Conv2d.apply(dt_, wt, 2, tpad, (h, w))
                if need[0]:
                    dx = dxs * s_
                if need[1]:
                    ds = _cg.dot_hw(dxs, x)
            if need[2] and not _cg.weight_gradients_disabled:
                dw = _cg._WGrad.apply(xs, dt_, (kh, kw), 2, tpad).transpose(0, 1)
        cast = lambda g, ref: g.to(ref.dtype) if (g is not None and ref is not None) else g
        return (dx, cast(ds, styles), cast(dw, weight), cast(dd, dcoefs), cast(dn, noise), cast(db, bias),
                None, None, None, None)


class _UpLayerVJP(torch.autograd.Function):
    """_LayerVJP for the up-2 layer (c = FIR(convT_s2(x * s, W)) * 4, z = act(c * d + noise + b) * gain), the
    path-length pass's other layer form.  With F the 4x4 FIR and L_W the stride-2 transposed conv:
        forward    dc = act'(dy; y) * d, dd = sum_hw act'(dy; y) * c                 (sg2_layer_bwd)
                   u = F^T dc (adjoint FIR), dxs = L_W^T u; dx = dxs * s, ds = sum_hw dxs * x   (one dgrad launch)
        backward   G = g_dx * s + g_ds * x
                   A d = F(L_W G) * d  (the layer's own forward on G: up-2 conv + FIR with the d scale)
                   g_dy = act'(A d + g_dd * c; y),  g_d = sum_hw (A d) * dc / d^2
                   H = g_dd * act'(dy; y) = dc * g_dd / d, and F^T H = u * g_dd / d (F is per channel), so
                   g_x = g_ds * dxs + L_W^T(u * g_dd / d) * s, g_s = sum g_dx * dxs + sum L_W^T(u * g_dd / d) * x
                   g_W = wgrad(G, u) + wgrad(x * s, u * g_dd / d)
    (reference: modulated_conv2d's up path, networks_stylegan2.py:66-76, through conv2d_resample.py:112-129)."""

    @staticmethod
    def forward(ctx, dy, x, styles, weight, dcoefs, y, c, f, need_x, need_s, need_d, alpha, gain, clamp, tpad,
                t_hw, fpad):
        n, cin, h, w = x.shape
        kh, kw = weight.shape[2], weight.shape[3]
        dt = x.dtype
        d32, s32 = _f32(dcoefs), _f32(styles)
        oh, ow = y.shape[2], y.shape[3]
        aup, adown, apad, aflip = _up.adjoint_params(f, t_hw, (oh, ow), 1, 1, fpad, False)
        dc, _, dd, _ = _cg.layer_bwd(dy.to(dt), y, c if need_d else None, d32, act=1, alpha=alpha, gain=gain,
                                     clamp=clamp, want_db=False, want_dd=need_d, want_dnoise=False)
        u = _up.upfirdn2d(dc, f, up=aup, down=adown, padding=apad, flip_filter=aflip, gain=4)
        wT = _cg._pack_conv(weight.transpose(0, 1), dt)
        if _cg._halo_s2_ok(u, kh, kw, 2, tpad, dot=need_s):
            dx, dxs, ds = _cg.conv3x3_fused(u, wT, cin, out_scale=s32, dot_src=x if need_s else None, stride=2,
                                            want_raw=True) + ((None,) if not need_s else ())
        else:
            res = _cg.conv_fused(u, wT, cin, h, w, kh, kw, 2, tpad, out_scale=s32, dot_src=x if need_s else None,
                                 aux_mode=1)
            dx, dxs, ds = res if need_s else res + (None,)
        ctx.save_for_backward(x, styles, weight, dcoefs, y, c, f, dc, u, dxs)
        ctx.cfg = (alpha, gain, clamp, tpad, t_hw, fpad)
        return (dx if need_x else None, ds.to(styles.dtype) if need_s else None,
                dd.to(dcoefs.dtype) if need_d else None)

    @staticmethod
    def backward(ctx, g_dx, g_ds, g_dd):
        if torch.is_grad_enabled():
            raise RuntimeError('_UpLayerVJP: third-order gradients are not supported (set modconv.fused_vjp = False)')
        x, styles, weight, dcoefs, y, c, f, dc, u, dxs = ctx.saved_tensors
        alpha, gain, clamp, tpad, (th, tw), fpad = ctx.cfg
        need = ctx.needs_input_grad
        n, cin, h, w = x.shape
        cout, _, kh, kw = weight.shape
        dt = x.dtype
        d32, s32 = _f32(dcoefs), _f32(styles)
        g_dy = g_x = g_s = g_w = g_d = None
        gds32 = _f32(g_ds)
        G = None
        if g_dx is not None:   # G = g_dx * s + g_ds * x and sum_p g_dx * dxs in one pass
            G, g_s = _cg.vjp_axpy(g_dx.to(dt), s32, x if g_ds is not None else None, gds32,
                                  e=dxs if need[2] else None)
        elif g_ds is not None:
            G, _ = _cg.vjp_axpy(x, gds32)
        hscale = (g_dd.float() / d32).contiguous() if g_dd is not None else None
        if G is not None and (need[0] or need[4]):
            tG, _ = _cg.conv_fused(G, _cg._pack_conv(weight, dt), cout, th, tw, kh, kw, 2, tpad, transpose=True)
            A_d, _ = _up.fir_fused(tG, f, fpad, gain=4.0, out_scale=d32)
            if need[4]:
                g_d = (_cg.dot_hw(A_d, dc) / (d32 * d32)).to(dcoefs.dtype)
            if need[0]:
                g_dy, _ = _cg.vjp_axpy(A_d, None, c if hscale is not None else None, _f32(g_dd) if hscale is not None
                                       else None, y=y, act=1, alpha=alpha, gain=gain, clamp=clamp)
        elif need[0] and hscale is not None:
            g_dy, _ = _cg.vjp_axpy(c, _f32(g_dd), y=y, act=1, alpha=alpha, gain=gain, clamp=clamp)
        if need[1] or need[2]:
            gxc = None
            if hscale is not None:
                wT = _cg._pack_conv(weight.transpose(0, 1), dt)
                dot_src = x if need[2] else None
                if _cg._halo_s2_ok(u, kh, kw, 2, tpad, dot=need[2]):
                    res = _cg.conv3x3_fused(u, wT, cin, in_scale=hscale, out_scale=s32, dot_src=dot_src, stride=2)
                else:
                    res = _cg.conv_fused(u, wT, cin, h, w, kh, kw, 2, tpad, in_scale=hscale, out_scale=s32,
                                         dot_src=dot_src)
                gxc = res[0]
                if need[2]:
                    g_s = res[2] if g_s is None else g_s + res[2]
            if need[1]:
                if g_ds is not None:
                    g_x, _ = (_cg.vjp_axpy(gxc, None, dxs, gds32) if gxc is not None else _cg.vjp_axpy(dxs, gds32))
                else:
                    g_x = gxc
        if need[3] and (G is not None or hscale is not None):
            acc = torch.zeros([cin * kh * kw * cout], dtype=torch.float32, device=x.device)
            # (the transposed conv's weight: the [cin, cout] gradient transposed, written so where the library can)
            if G is not None:
                g_w = _cg._wgrad_raw(G, u, kh, kw, 2, tpad, out=acc, param_layout='swap')
            if hscale is not None:
                g_w = _cg._wgrad_raw(x, u, kh, kw, 2, tpad, g_scale=s32, x_scale=hscale, out=acc, param_layout='swap')
            g_w = g_w.transpose(0, 1).to(weight.dtype)
        g_s = g_s.to(styles.dtype) if g_s is not None else None
        return (g_dy, g_x, g_s, g_w, g_d) + (None,) * 12


def up_modconv_layer(x, styles, weight, dcoefs, noise, bias, f, alpha, gain, clamp):
    return UpModConv.apply(x, styles, weight, dcoefs, noise, bias, f, float(alpha), float(gain),
                           float(clamp if clamp is not None else -1.0))
