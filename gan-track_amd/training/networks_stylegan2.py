"""StyleGAN2 generator and discriminator on the MI355X kernels.

Drop-in for SG3/training/networks_stylegan2.py: same classes, constructor arguments, forward
signatures and parameter/buffer names (`synthesis.b256.conv1.weight`, `mapping.fc0.weight`,
`mapping.w_avg`, ...), so state dicts and `copy_params_and_buffers` interoperate.

MI355X-specific execution choices (numerically equivalent to the reference up to rounding):
  * feature maps live in NHWC memory (torch.channels_last) end to end -- the layout the MFMA
    implicit-GEMM convolutions consume; 1-channel images are layout-agnostic;
  * blocks at the `num_fp16_res` highest resolutions compute in float16 (the reference's choice,
    :474-486) or in bfloat16 when `fp16_dtype=torch.bfloat16`;
  * modulated_conv2d always scales activations around one shared convolution
    (`x*s -> conv -> x*d + noise`); the reference's grouped "fused" form (:79-89) is the same
    contraction regrouped (verified equal to 7e-15 in fp64) and is computed this way;
  * demodulation uses sum_i s_i^2 * sum_k W_oik^2 -- no [N,O,I,k,k] temporary.
"""
import numpy as np
import torch

import sg2hip as _hip
from torch_utils import misc
from torch_utils import persistence
from torch_utils.ops import bias_act
from torch_utils.ops import conv2d_gradfix
from torch_utils.ops import conv2d_resample
from torch_utils.ops import fma
from torch_utils.ops import modconv
from torch_utils.ops import staged_sum
from torch_utils.ops import upfirdn2d

_CL = torch.channels_last


def normalize_2nd_moment(x, dim=1, eps=1e-8):
    """:26-27"""
    return x * (x.square().mean(dim=dim, keepdim=True) + eps).rsqrt()


class _InfNorm(torch.autograd.Function):
    """fp16 range pre-normalisation (:52-54), row-wise over t [rows, L]: mode 0 is the weight,
    t * (c / max|t|) with c = 1/sqrt(fan_in); mode 1 the styles, t / max|t|.  One kernel forward
    (sg2_infnorm_fwd) and one first-order backward (sg2_infnorm_bwd) in place of the ~20 launches of the
    composed norm / reciprocal / scale / multiply and their autograd.  Under create_graph (the path-length
    pass) the backward re-derives the reference expression with autograd so that second-order terms exist."""

    @staticmethod
    def forward(ctx, t_in, c, mode):
        t = t_in.contiguous()
        rows, L = t.shape
        y = torch.empty_like(t)
        nrm = torch.empty([rows], dtype=torch.float32, device=t.device)
        _hip.check(_hip.lib().sg2_infnorm_fwd(_hip.ptr(y), _hip.ptr(nrm), _hip.ptr(t), rows, L, float(c), mode,
                                              _hip.stream_ptr(t.device)), 'sg2_infnorm_fwd')
        ctx.save_for_backward(t_in, nrm)    # the input itself: the create_graph backward differentiates it
        ctx.c, ctx.mode = c, mode
        return y

    @staticmethod
    def backward(ctx, dy):
        t, nrm = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None
        if torch.is_grad_enabled():
            return _InfNormVJP.apply(dy, t, nrm, ctx.c if ctx.mode == 0 else 1.0, ctx.mode), None, None
        dy, t = dy.contiguous(), t.contiguous()
        dt = torch.empty_like(t)
        _hip.check(_hip.lib().sg2_infnorm_bwd(_hip.ptr(dt), _hip.ptr(dy), _hip.ptr(t), _hip.ptr(nrm), t.shape[0],
                                              t.shape[1], float(ctx.c), ctx.mode, _hip.stream_ptr(t.device)),
                   'sg2_infnorm_bwd')
        return dt, None, None


class _InfNormVJP(torch.autograd.Function):
    """The first-order gradient of _InfNorm as ONE differentiable node (the path-length pass differentiates it once
    more): forward dt = c dy / n - c P e / n^2 (sg2_infnorm_bwd), with n = max_j |t_j| per row, P = sum_j dy_j t_j and
    e_j = sign(t_j) [|t_j| = n] / (number of maxima) -- torch's infinity-norm gradient, ties split evenly; backward
    from the closed form (the maxima mask piecewise constant):
        g_dy = c (g - t (g.e) / n) / n
        g_t  = c (2 P (g.e) e / n^3 - ((g.dy) e + (g.e) dy) / n^2)
    in one launch (sg2_infnorm_vjp_bwd), where autograd of the reference expression re-derived under create_graph
    (norm, reciprocal, scale, multiply) and differentiated again ran ~40 per call (tests/test_ops_gpu.py::
    test_infnorm_prenorm checks the second order against it)."""

    @staticmethod
    def forward(ctx, dy, t, nrm, c, mode):
        dy, t = dy.contiguous(), t.contiguous()
        dt = torch.empty_like(t)
        _hip.check(_hip.lib().sg2_infnorm_bwd(_hip.ptr(dt), _hip.ptr(dy), _hip.ptr(t), _hip.ptr(nrm), t.shape[0],
                                              t.shape[1], float(c), mode, _hip.stream_ptr(t.device)), 'sg2_infnorm_bwd')
        ctx.save_for_backward(dy, t, nrm)
        ctx.c = c
        return dt

    @staticmethod
    def backward(ctx, g):
        dy, t, nrm = ctx.saved_tensors
        g = g.float().contiguous()
        g_dy = torch.empty_like(dy) if ctx.needs_input_grad[0] else None
        g_t = torch.empty_like(t) if ctx.needs_input_grad[1] else None
        _hip.check(_hip.lib().sg2_infnorm_vjp_bwd(_hip.ptr(g_dy), _hip.ptr(g_t), _hip.ptr(g), _hip.ptr(dy),
                                                  _hip.ptr(t), _hip.ptr(nrm), t.shape[0], t.shape[1], float(ctx.c),
                                                  _hip.stream_ptr(t.device)), 'sg2_infnorm_vjp_bwd')
        return g_dy, g_t, None, None, None


def _prenorm(weight, styles):
    """(:52-54) weight * (1/sqrt(I*k*k) / ||weight||_inf per output channel), styles / ||styles||_inf per sample."""
    o, i, kh, kw = weight.shape
    if weight.dtype != torch.float32 or styles.dtype != torch.float32:
        return (weight * (1 / np.sqrt(i * kh * kw) / weight.norm(float('inf'), dim=[1, 2, 3], keepdim=True)),
                styles / styles.norm(float('inf'), dim=1, keepdim=True))
    w = _InfNorm.apply(weight.reshape(o, -1), float(np.float32(1 / np.sqrt(i * kh * kw))), 0).reshape(o, i, kh, kw)
    return w, _InfNorm.apply(styles, 1.0, 1)


class _Demod(torch.autograd.Function):
    """d[n,o] = rsqrt(sum_i s[n,i]^2 sum_k w[o,i,k]^2 + 1e-8) in one kernel (sg2_demod_fwd) where autograd
    of the reference's expression (:59-63) runs six elementwise / reduction / GEMM launches, and the
    first-order gradient in two (sg2_demod_bwd).  Under create_graph (the path-length pass) the gradient
    is composed of differentiable torch ops."""

    @staticmethod
    def forward(ctx, weight, styles):
        w = weight.float().contiguous()
        s = styles.float().contiguous()
        n, o, i, kk = s.shape[0], w.shape[0], w.shape[1], w.shape[2] * w.shape[3]
        d = torch.empty([n, o], dtype=torch.float32, device=s.device)
        wsq = torch.empty([o, i], dtype=torch.float32, device=s.device)
        _hip.check(_hip.lib().sg2_demod_fwd(_hip.ptr(d), _hip.ptr(wsq), _hip.ptr(s), _hip.ptr(w), n, o, i, kk, 1e-8,
                                            _hip.stream_ptr(s.device)), 'sg2_demod_fwd')
        ctx.save_for_backward(w, s, d, wsq)
        return d

    @staticmethod
    def backward(ctx, dd):
        w, s, d, wsq = ctx.saved_tensors
        need_w, need_s = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if torch.is_grad_enabled():
            # Inside no_weight_gradients (the path-length / R1 first pass, which asks autograd.grad for the latent
            # or image gradient only) the weight's gradient is never used: autograd's engine would prune it for
            # the reference's composed expression; a custom Function's needs_input_grad cannot tell, so skip it
            # here instead of building its double-backward graph.
            need_w = need_w and not conv2d_gradfix.weight_gradients_disabled
            if need_s and not need_w:
                return None, _DemodVJP.apply(dd, d, w, s, wsq)
            gu = dd * d.pow(3) * -0.5
            gs = 2 * s * (gu @ w.square().sum([2, 3])) if need_s else None
            gw = 2 * w * (gu.t() @ s.square())[:, :, None, None] if need_w else None
            return gw, gs
        dd = dd.float().contiguous()
        n, o, i, kk = s.shape[0], w.shape[0], w.shape[1], w.shape[2] * w.shape[3]
        gw = torch.empty_like(w) if need_w else None
        gs = torch.empty_like(s) if need_s else None
        _hip.check(_hip.lib().sg2_demod_bwd(_hip.ptr(gs), _hip.ptr(gw), _hip.ptr(dd), _hip.ptr(d), _hip.ptr(s),
                                            _hip.ptr(w), _hip.ptr(wsq), n, o, i, kk, _hip.stream_ptr(s.device)),
                   'sg2_demod_bwd')
        return gw, gs


class _DemodVJP(torch.autograd.Function):
    """The styles' gradient of _Demod as one differentiable node for the path-length pass (whose first pass wants
    no weight gradient): forward gs = 2 s (u @ wsq) with u = -dd d^3 / 2 and wsq = sum_k w^2 (sg2_demod_bwd, one
    launch where the composed form runs seven); backward from the closed form in two (sg2_demod_vjp_bwd)
        g_s = 2 G (u @ wsq),  g_u = (2 s G) @ wsq^T,  g_w = 2 w (u^T @ (2 s G)),
        g_dd = -d^3 g_u / 2,  g_d = -3 dd d^2 g_u / 2
    (d, w and s carry their own autograd history, so the second pass continues into _Demod, the weight and the
    styles exactly as the composed expression did)."""

    @staticmethod
    def forward(ctx, dd, d, w, s, wsq):
        dd = dd.float().contiguous()
        n, o, i, kk = s.shape[0], w.shape[0], w.shape[1], w.shape[2] * w.shape[3]
        gs = torch.empty_like(s)
        _hip.check(_hip.lib().sg2_demod_bwd(_hip.ptr(gs), _hip.ptr(None), _hip.ptr(dd), _hip.ptr(d), _hip.ptr(s), _hip.ptr(w),
                                            _hip.ptr(wsq), n, o, i, kk, _hip.stream_ptr(s.device)), 'sg2_demod_bwd')
        ctx.save_for_backward(dd, d, w, s, wsq)
        return gs

    @staticmethod
    def backward(ctx, g):
        dd, d, w, s, wsq = ctx.saved_tensors
        g = g.float().contiguous()
        need = ctx.needs_input_grad
        g_dd = torch.empty_like(dd) if need[0] else None
        g_d = torch.empty_like(d) if need[1] else None
        g_w = torch.empty_like(w) if need[2] else None
        g_s = torch.empty_like(s) if need[3] else None
        n, o, i, kk = s.shape[0], w.shape[0], w.shape[1], w.shape[2] * w.shape[3]
        _hip.check(_hip.lib().sg2_demod_vjp_bwd(_hip.ptr(g_dd), _hip.ptr(g_d), _hip.ptr(g_w), _hip.ptr(g_s),
                                                _hip.ptr(g), _hip.ptr(dd), _hip.ptr(d), _hip.ptr(s), _hip.ptr(w),
                                                _hip.ptr(wsq), n, o, i, kk, _hip.stream_ptr(s.device)),
                   'sg2_demod_vjp_bwd')
        return g_dd, g_d, g_w, g_s, None


def _demod(weight, styles):
    """d[n,o] = rsqrt(sum_i s[n,i]^2 sum_k w[o,i,k]^2 + 1e-8)   (:59-63, regrouped)."""
    if weight.shape[1] <= 1024 and weight.shape[0] <= 1024 and styles.shape[0] <= 1024:
        return _Demod.apply(weight, styles)
    wsq = weight.float().square().sum(dim=[2, 3])                 # [O, I]
    return (styles.float().square() @ wsq.t() + 1e-8).rsqrt()     # [N, O]


def modulated_conv2d(x, weight, styles, noise=None, up=1, down=1, padding=0, resample_filter=None,
                     demodulate=True, flip_weight=True, fused_modconv=True):
    """Weight-modulated convolution (:32-89).  x [N,I,H,W], weight [O,I,k,k], styles [N,I]."""
    n = x.shape[0]
    out_ch, in_ch, kh, kw = weight.shape
    misc.assert_shape(weight, [out_ch, in_ch, kh, kw])
    misc.assert_shape(x, [n, in_ch, None, None])
    misc.assert_shape(styles, [n, in_ch])
    if x.dtype == torch.float16 and demodulate:   # keep fp16 in range (:52-54)
        weight, styles = _prenorm(weight, styles)
    dcoefs = _demod(weight, styles) if demodulate else None
    x = x * styles.to(x.dtype).reshape(n, -1, 1, 1)
    x = conv2d_resample.conv2d_resample(x=x, w=weight.to(x.dtype), f=resample_filter, up=up, down=down,
                                        padding=padding, flip_weight=flip_weight)
    if demodulate and noise is not None:
        return fma.fma(x, dcoefs.to(x.dtype).reshape(n, -1, 1, 1), noise.to(x.dtype))
    if demodulate:
        return x * dcoefs.to(x.dtype).reshape(n, -1, 1, 1)
    if noise is not None:
        return x + noise.to(x.dtype)
    return x


class _Addmm(torch.autograd.Function):
    """y = beta * b + alpha * x @ w^T with the scalars kept inside the GEMMs of the first-order backward too
    (dx = alpha dy @ w, dw = alpha dy^T x as beta = 0 addmms; autograd of torch.addmm runs a GEMM and a
    separate scale for each).  Under create_graph (the path-length pass through the affine layers) the
    backward is built from differentiable ops."""

    @staticmethod
    def forward(ctx, b, x, w, beta, alpha):
        ctx.save_for_backward(x, w)
        ctx.beta, ctx.alpha = beta, alpha
        return torch.addmm(b, x, w.t(), beta=beta, alpha=alpha)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        beta, alpha = ctx.beta, ctx.alpha
        nb, nx, nw = ctx.needs_input_grad[:3]
        if torch.is_grad_enabled():
            pg = not conv2d_gradfix.weight_gradients_disabled   # (see _Demod.backward: parameter grads unused)
            return ((dy.sum(0) * beta) if nb and pg else None, (dy @ w) * alpha if nx else None,
                    (dy.t() @ x) * alpha if nw and pg else None, None, None)
        z = _zero_scalar(dy)
        db = None
        if nb:   # beta * sum_rows(dy) as ONE GEMV (a sum and a scale otherwise)
            db = torch.addmv(_zero_vec(dy, dy.shape[1]), dy.t(), _ones(dy, dy.shape[0]), beta=0, alpha=beta) \
                if beta != 1 else dy.sum(0)
        dx = torch.addmm(z, dy, w, beta=0, alpha=alpha) if nx else None
        dw = torch.addmm(z, dy.t(), x, beta=0, alpha=alpha) if nw else None
        return db, dx, dw, None, None


def _zero_scalar(t):
    return torch.empty((), dtype=t.dtype, device=t.device)   # beta = 0: never read


def _zero_vec(t, n):
    return torch.empty((n,), dtype=t.dtype, device=t.device)  # beta = 0: never read


_ONES = {}


def _ones(t, n):
    key = (n, t.dtype, t.device)
    v = _ONES.get(key)
    if v is None:
        v = _ONES[key] = torch.ones(n, dtype=t.dtype, device=t.device)
    return v


@persistence.persistent_class
class FullyConnectedLayer(torch.nn.Module):
    """:94-125"""

    def __init__(self, in_features, out_features, bias=True, activation='linear', lr_multiplier=1, bias_init=0):
        super().__init__()
        self.in_features, self.out_features, self.activation = in_features, out_features, activation
        self.weight = torch.nn.Parameter(torch.randn([out_features, in_features]) / lr_multiplier)
        self.bias = torch.nn.Parameter(torch.full([out_features], np.float32(bias_init))) if bias else None
        self.weight_gain = lr_multiplier / np.sqrt(in_features)
        self.bias_gain = lr_multiplier

    def forward(self, x, out_gain=1):
        """y = act(x @ (W * weight_gain)^T + b * bias_gain) (* out_gain for a linear layer).  The weight and
        bias gains (reference :111-125: two elementwise multiplies per call, and their backward) are the
        alpha / beta scalars of ONE addmm; `out_gain` folds ToRGBLayer's styles * weight_gain (:352)."""
        w = self.weight if self.weight.dtype == x.dtype else self.weight.to(x.dtype)
        b = self.bias
        if b is not None:
            b = b if b.dtype == x.dtype else b.to(x.dtype)
            if self.activation == 'linear':
                return _Addmm.apply(b, x, w, float(self.bias_gain * out_gain), float(self.weight_gain * out_gain))
            y = _Addmm.apply(b, x, w, float(self.bias_gain), float(self.weight_gain))
            return bias_act.bias_act(y, None, act=self.activation)
        y = x.matmul((w * (self.weight_gain * out_gain)).t())
        return bias_act.bias_act(y, None, act=self.activation) if self.activation != 'linear' else y

    def extra_repr(self):
        return f'in_features={self.in_features:d}, out_features={self.out_features:d}, activation={self.activation:s}'


# The synthesis network's affine layers (one FullyConnectedLayer per conv / toRGB layer, 20 at 256^2) as ONE
# GEMM: every layer's weight rows side by side, every w row against all of them (S = ws @ W_cat^T, N * num_ws x
# sum C -- the off-diagonal blocks are wasted but cost microseconds), then one gather picks each layer's block
# (its w row, its columns) into a layer-major buffer whose per-layer slices are contiguous [N, C], with the
# layer's weight / bias gains.  The bias rows enter through a rank-1 GEMM (ones[N] x b * gain) gathered with
# unique indices, so the backward has no duplicate-index scatter (whose atomics would make the bias gradients
# run-to-run different; sg2hip.deterministic).  Autograd of these few torch ops (mm, take, addcmul, cat) replaces ~3 launches per
# layer forward and ~4 backward (GEMMs, GEMVs, the ws unbind / narrow adds), and is differentiable twice (the
# path-length pass).  Reference per layer: networks_stylegan2.py:111-125 (styles = affine(w)), :352 (toRGB's
# styles * weight_gain).
grouped_affine = True
_PLAN_CACHE = {}


def _style_plan(layers, n, num_ws, device):
    """Index / gain tensors of grouped_styles for one batch size: (elem index into S, elem index into the
    [N, sum C] bias matrix, elem alpha, column beta, ones [N, 1], per-layer (offset, C)).  The plan is a pure
    function of each layer's width, gains, w index and out gain (no module identity in the key: ids are reused
    once a network is freed)."""
    key = (tuple((int(a.out_features), float(a.weight_gain), float(a.bias_gain), int(k), float(g)) for a, k, g in layers),
           n, num_ws, str(device))
    plan = _PLAN_CACHE.get(key)
    if plan is not None:
        return plan
    tot = sum(a.out_features for a, _, _ in layers)
    idx, bidx, alpha, beta, spans = [], [], [], [], []
    col, off = 0, 0
    for a, k, g in layers:
        c = a.out_features
        rows = np.arange(n)[:, None] * num_ws + k                      # [N, 1]
        cols = col + np.arange(c)[None, :]                             # [1, C]
        idx.append((rows * tot + cols).reshape(-1))
        bidx.append((np.arange(n)[:, None] * tot + cols).reshape(-1))
        alpha.append(np.full(n * c, np.float32(a.weight_gain * g), np.float32))
        beta.append(np.full(c, np.float32(a.bias_gain * g), np.float32))
        spans.append((off, c))
        col += c
        off += n * c
    T = lambda v, dt: torch.as_tensor(np.concatenate(v), dtype=dt, device=device)  # noqa: E731
    plan = (T(idx, torch.int64), T(bidx, torch.int64), T(alpha, torch.float32), T(beta, torch.float32),
            torch.ones([n, 1], dtype=torch.float32, device=device), spans)
    _PLAN_CACHE[key] = plan
    return plan


def grouped_styles(ws, layers):
    """ws [N, num_ws, w_dim] f32; layers: [(FullyConnectedLayer (linear, with bias), w index, out gain)] ->
    per-layer styles [N, C] (contiguous) = ws[:, k] @ (W * weight_gain)^T * g + b * bias_gain * g."""
    n, num_ws, d = ws.shape
    W = torch.cat([a.weight for a, _, _ in layers])
    b = torch.cat([a.bias for a, _, _ in layers])
    S = torch.mm(ws.reshape(n * num_ws, d), W.t())
    idx, bidx, alpha, beta, ones, spans = _style_plan(layers, n, num_ws, ws.device)
    B = torch.mm(ones, (b * beta).view(1, -1))                         # [N, sum C]: row n = b * gain
    out = torch.addcmul(B.take(bidx), S.take(idx), alpha)
    # split (not narrow): its backward is ONE cat of the layers' gradients, a narrow's is a zero-filled full-size
    # slice_backward per layer plus the adds that sum them
    return [t.view(n, c) for t, (_, c) in zip(out.split([n * c for _, c in spans]), spans)]


@persistence.persistent_class
class Conv2dLayer(torch.nn.Module):
    """:133-181"""

    def __init__(self, in_channels, out_channels, kernel_size, bias=True, activation='linear', up=1, down=1,
                 resample_filter=[1, 3, 3, 1], conv_clamp=None, channels_last=False, trainable=True):
        super().__init__()
        self.in_channels, self.out_channels, self.activation = in_channels, out_channels, activation
        self.up, self.down, self.conv_clamp = up, down, conv_clamp
        self.register_buffer('resample_filter', upfirdn2d.setup_filter(resample_filter))
        self.padding = kernel_size // 2
        self.weight_gain = 1 / np.sqrt(in_channels * (kernel_size ** 2))
        self.act_gain = bias_act.activation_funcs[activation].def_gain
        weight = torch.randn([out_channels, in_channels, kernel_size, kernel_size])
        bias = torch.zeros([out_channels]) if bias else None
        if trainable:
            self.weight = torch.nn.Parameter(weight)
            self.bias = torch.nn.Parameter(bias) if bias is not None else None
        else:
            self.register_buffer('weight', weight)
            if bias is not None:
                self.register_buffer('bias', bias)
            else:
                self.bias = None

    def forward(self, x, gain=1, residual=None, prefiltered=False):
        """residual (DiscriminatorBlock's resnet skip, :621-627) is added to the activated output.
        prefiltered: a 1x1 down-2 layer's input already went through its FIR (upfirdn2d.fork_fir)."""
        clamp = self.conv_clamp * gain if self.conv_clamp is not None else None
        kh = self.weight.shape[2]
        if self.activation in ('lrelu', 'linear') and self.up == 1 and modconv.supported_generic(x, self.weight):
            # conv + bias + act + gain + clamp (+ residual) in one kernel; the FIR of a down-2 layer runs
            # first (conv2d_resample.py:94-97 / :106-109 plans, same padding algebra)
            stride, pad = 1, self.padding
            if self.down > 1:
                x0, x1, y0, y1 = conv2d_resample._frame_padding(self.padding, self.resample_filter, 1, self.down)
                if kh == 1:
                    if not prefiltered:
                        x = upfirdn2d.upfirdn2d(x, self.resample_filter, down=self.down, padding=[x0, x1, y0, y1])
                else:
                    x = upfirdn2d.upfirdn2d(x, self.resample_filter, padding=[x0, x1, y0, y1])
                    stride = self.down
                pad = 0
            # the weight gain (`w = self.weight * self.weight_gain`, :173) rides in the weight pack and the
            # weight-gradient kernel: no elementwise launch forward or backward
            return modconv.fused_conv(x, self.weight, bias=self.bias, residual=residual, stride=stride, padding=pad,
                                      act=self.activation, alpha=bias_act.activation_funcs[self.activation].def_alpha or 0.2,
                                      gain=self.act_gain * gain, clamp=clamp, wgain=self.weight_gain)
        w = self.weight * self.weight_gain
        b = self.bias.to(x.dtype) if self.bias is not None else None
        pre = prefiltered and self.down > 1 and kh == 1
        x = conv2d_resample.conv2d_resample(x=x, w=w.to(x.dtype), f=None if pre else self.resample_filter, up=self.up,
                                            down=1 if pre else self.down, padding=self.padding,
                                            flip_weight=(self.up == 1))
        x = bias_act.bias_act(x, b, act=self.activation, gain=self.act_gain * gain, clamp=clamp)
        return x if residual is None else residual.add_(x)

    def extra_repr(self):
        return (f'in_channels={self.in_channels:d}, out_channels={self.out_channels:d}, '
                f'activation={self.activation:s}, up={self.up}, down={self.down}')


@persistence.persistent_class
class MappingNetwork(torch.nn.Module):
    """:191-269"""

    def __init__(self, z_dim, c_dim, w_dim, num_ws, num_layers=8, embed_features=None, layer_features=None,
                 activation='lrelu', lr_multiplier=0.01, w_avg_beta=0.998):
        super().__init__()
        self.z_dim, self.c_dim, self.w_dim, self.num_ws = z_dim, c_dim, w_dim, num_ws
        self.num_layers, self.w_avg_beta = num_layers, w_avg_beta
        if embed_features is None:
            embed_features = w_dim
        if c_dim == 0:
            embed_features = 0
        if layer_features is None:
            layer_features = w_dim
        feats = [z_dim + embed_features] + [layer_features] * (num_layers - 1) + [w_dim]
        if c_dim > 0:
            self.embed = FullyConnectedLayer(c_dim, embed_features)
        for idx in range(num_layers):
            setattr(self, f'fc{idx}', FullyConnectedLayer(feats[idx], feats[idx + 1], activation=activation,
                                                          lr_multiplier=lr_multiplier))
        if num_ws is not None and w_avg_beta is not None:
            self.register_buffer('w_avg', torch.zeros([w_dim]))

    def forward(self, z, c, truncation_psi=1, truncation_cutoff=None, update_emas=False):
        x = None
        if self.z_dim > 0:
            misc.assert_shape(z, [None, self.z_dim])
            x = normalize_2nd_moment(z.to(torch.float32))
        if self.c_dim > 0:
            misc.assert_shape(c, [None, self.c_dim])
            y = normalize_2nd_moment(self.embed(c.to(torch.float32)))
            x = torch.cat([x, y], dim=1) if x is not None else y
        for idx in range(self.num_layers):
            x = getattr(self, f'fc{idx}')(x)
        if update_emas and self.w_avg_beta is not None:
            self.w_avg.copy_(x.detach().mean(dim=0).lerp(self.w_avg, self.w_avg_beta))
        if self.num_ws is not None:
            x = x.unsqueeze(1).repeat([1, self.num_ws, 1])
        if truncation_psi != 1:
            assert self.w_avg_beta is not None
            if self.num_ws is None or truncation_cutoff is None:
                x = self.w_avg.lerp(x, truncation_psi)
            else:
                x[:, :truncation_cutoff] = self.w_avg.lerp(x[:, :truncation_cutoff], truncation_psi)
        return x

    def extra_repr(self):
        return f'z_dim={self.z_dim:d}, c_dim={self.c_dim:d}, w_dim={self.w_dim:d}, num_ws={self.num_ws}'


@persistence.persistent_class
class SynthesisLayer(torch.nn.Module):
    """:273-333"""

    def __init__(self, in_channels, out_channels, w_dim, resolution, kernel_size=3, up=1, use_noise=True,
                 activation='lrelu', resample_filter=[1, 3, 3, 1], conv_clamp=None, channels_last=False):
        super().__init__()
        self.in_channels, self.out_channels, self.w_dim = in_channels, out_channels, w_dim
        self.resolution, self.up, self.use_noise = resolution, up, use_noise
        self.activation, self.conv_clamp = activation, conv_clamp
        self.register_buffer('resample_filter', upfirdn2d.setup_filter(resample_filter))
        self.padding = kernel_size // 2
        self.act_gain = bias_act.activation_funcs[activation].def_gain
        self.affine = FullyConnectedLayer(w_dim, in_channels, bias_init=1)
        self.weight = torch.nn.Parameter(torch.randn([out_channels, in_channels, kernel_size, kernel_size]))
        if use_noise:
            self.register_buffer('noise_const', torch.randn([resolution, resolution]))
            self.noise_strength = torch.nn.Parameter(torch.zeros([]))
        self.bias = torch.nn.Parameter(torch.zeros([out_channels]))

    def forward(self, x, w, noise_mode='random', fused_modconv=True, gain=1, styles=None):
        """styles: this layer's affine(w), when the network computed it (grouped_styles)."""
        assert noise_mode in ['random', 'const', 'none']
        misc.assert_shape(x, [None, self.in_channels, self.resolution // self.up, self.resolution // self.up])
        if styles is None:
            styles = self.affine(w)
        noise = None
        if self.use_noise and noise_mode == 'random':
            noise = staged_sum.scale_by_scalar(torch.randn([x.shape[0], 1, self.resolution, self.resolution],
                                                           device=x.device), self.noise_strength)
        if self.use_noise and noise_mode == 'const':
            noise = staged_sum.scale_by_scalar(self.noise_const, self.noise_strength)
        up_fused = self.up == 2 and modconv.supported_up(x, self.weight, self.resample_filter)
        if self.activation == 'lrelu' and (up_fused or (self.up == 1 and modconv.supported_generic(x, self.weight))):
            # one-kernel modulated conv + demod + noise + bias + lrelu + clamp (sg2_conv3x3 / sg2_conv2d_fused)
            weight = self.weight
            if x.dtype == torch.float16:   # fp16 range pre-normalisation (:52-54)
                weight, styles = _prenorm(weight, styles)
            if noise is not None and noise.ndim == 2:
                noise = noise.reshape(1, 1, *noise.shape).expand(x.shape[0], 1, -1, -1)
            clamp = self.conv_clamp * gain if self.conv_clamp is not None else None
            if up_fused:
                return modconv.up_modconv_layer(x, styles, weight, _demod(weight, styles), noise, self.bias,
                                                self.resample_filter,
                                                alpha=bias_act.activation_funcs[self.activation].def_alpha,
                                                gain=self.act_gain * gain, clamp=clamp)
            return modconv.modconv_layer(x, styles, weight, _demod(weight, styles), noise, self.bias,
                                         alpha=bias_act.activation_funcs[self.activation].def_alpha,
                                         gain=self.act_gain * gain, clamp=clamp)
        x = modulated_conv2d(x=x, weight=self.weight, styles=styles, noise=noise, up=self.up, padding=self.padding,
                             resample_filter=self.resample_filter, flip_weight=(self.up == 1),
                             fused_modconv=fused_modconv)
        clamp = self.conv_clamp * gain if self.conv_clamp is not None else None
        return bias_act.bias_act(x, self.bias.to(x.dtype), act=self.activation, gain=self.act_gain * gain, clamp=clamp)

    def extra_repr(self):
        return (f'in_channels={self.in_channels:d}, out_channels={self.out_channels:d}, w_dim={self.w_dim:d}, '
                f'resolution={self.resolution:d}, up={self.up}, activation={self.activation:s}')


@persistence.persistent_class
class ToRGBLayer(torch.nn.Module):
    """:337-358"""

    def __init__(self, in_channels, out_channels, w_dim, kernel_size=1, conv_clamp=None, channels_last=False):
        super().__init__()
        self.in_channels, self.out_channels, self.w_dim = in_channels, out_channels, w_dim
        self.conv_clamp = conv_clamp
        self.affine = FullyConnectedLayer(w_dim, in_channels, bias_init=1)
        self.weight = torch.nn.Parameter(torch.randn([out_channels, in_channels, kernel_size, kernel_size]))
        self.bias = torch.nn.Parameter(torch.zeros([out_channels]))
        self.weight_gain = 1 / np.sqrt(in_channels * (kernel_size ** 2))

    def forward(self, x, w, fused_modconv=True, styles=None):
        if styles is None:
            styles = self.affine(w, out_gain=self.weight_gain)
        if modconv.supported_generic(x, self.weight):
            # modulation folded into the conv's operand staging, bias + clamp into its epilogue
            return modconv.fused_conv(x, self.weight, styles=styles, bias=self.bias,
                                      padding=self.weight.shape[-1] // 2, clamp=self.conv_clamp)
        x = modulated_conv2d(x=x, weight=self.weight, styles=styles, demodulate=False, fused_modconv=fused_modconv)
        return bias_act.bias_act(x, self.bias.to(x.dtype), clamp=self.conv_clamp)

    def forward_tap(self, x, w, fused_modconv=True, styles=None):
        """(x, self(x, w)) for a feature map that also feeds the next block: its two gradients are added inside the
        toRGB input gradient's epilogue (modconv.FusedConvTap) instead of by autograd in an activation-sized pass."""
        if styles is None:
            styles = self.affine(w, out_gain=self.weight_gain)
        if modconv.tap_enabled and modconv.supported_generic(x, self.weight):
            return modconv.fused_conv_tap(x, self.weight, styles, self.bias, self.weight.shape[-1] // 2,
                                          self.conv_clamp)
        return x, self.forward(x, w, fused_modconv=fused_modconv, styles=styles)

    def extra_repr(self):
        return f'in_channels={self.in_channels:d}, out_channels={self.out_channels:d}, w_dim={self.w_dim:d}'


@persistence.persistent_class
class SynthesisBlock(torch.nn.Module):
    """:362-462"""

    def __init__(self, in_channels, out_channels, w_dim, resolution, img_channels, is_last, architecture='skip',
                 resample_filter=[1, 3, 3, 1], conv_clamp=256, use_fp16=False, fp16_channels_last=False,
                 fused_modconv_default=True, fp16_dtype=torch.float16, **layer_kwargs):
        assert architecture in ['orig', 'skip', 'resnet']
        super().__init__()
        self.in_channels, self.w_dim, self.resolution = in_channels, w_dim, resolution
        self.img_channels, self.is_last, self.architecture = img_channels, is_last, architecture
        self.use_fp16, self.fp16_dtype = use_fp16, fp16_dtype
        self.channels_last = True
        self.fused_modconv_default = fused_modconv_default
        self.register_buffer('resample_filter', upfirdn2d.setup_filter(resample_filter))
        self.num_conv = 0
        self.num_torgb = 0
        if in_channels == 0:
            self.const = torch.nn.Parameter(torch.randn([out_channels, resolution, resolution]))
        if in_channels != 0:
            self.conv0 = SynthesisLayer(in_channels, out_channels, w_dim=w_dim, resolution=resolution, up=2,
                                        resample_filter=resample_filter, conv_clamp=conv_clamp, **layer_kwargs)
            self.num_conv += 1
        self.conv1 = SynthesisLayer(out_channels, out_channels, w_dim=w_dim, resolution=resolution,
                                    conv_clamp=conv_clamp, **layer_kwargs)
        self.num_conv += 1
        if is_last or architecture == 'skip':
            self.torgb = ToRGBLayer(out_channels, img_channels, w_dim=w_dim, conv_clamp=conv_clamp)
            self.num_torgb += 1
        if in_channels != 0 and architecture == 'resnet':
            self.skip = Conv2dLayer(in_channels, out_channels, kernel_size=1, bias=False, up=2,
                                    resample_filter=resample_filter)

    def style_layers(self):
        """(affine, w index within the block's ws, out gain) of the block's layers in w order."""
        out, k = [], 0
        if self.in_channels != 0:
            out.append((self.conv0.affine, k, 1.0))
            k += 1
        out.append((self.conv1.affine, k, 1.0))
        k += 1
        if self.is_last or self.architecture == 'skip':
            out.append((self.torgb.affine, k, float(self.torgb.weight_gain)))
        return out

    def forward(self, x, img, ws, force_fp32=False, fused_modconv=None, update_emas=False, styles=None,
                **layer_kwargs):
        """styles: the layers' styles in w order (SynthesisNetwork's grouped_styles), or None (per-layer affine)."""
        misc.assert_shape(ws, [None, self.num_conv + self.num_torgb, self.w_dim])
        if styles is not None:
            s_iter = iter(styles)
            w_iter = iter([None] * len(styles))
        else:
            s_iter = iter([None] * (self.num_conv + self.num_torgb))
            w_iter = iter(ws.unbind(dim=1))
        dtype = self.fp16_dtype if self.use_fp16 and not force_fp32 else torch.float32
        if fused_modconv is None:
            fused_modconv = self.fused_modconv_default
        if fused_modconv == 'inference_only':
            fused_modconv = not self.training
        if self.in_channels == 0:
            x = self.const.to(dtype=dtype).unsqueeze(0).repeat([ws.shape[0], 1, 1, 1])
            x = x.contiguous(memory_format=_CL)
        else:
            misc.assert_shape(x, [None, self.in_channels, self.resolution // 2, self.resolution // 2])
            x = x.to(dtype=dtype, memory_format=_CL)
        if self.in_channels == 0:
            x = self.conv1(x, next(w_iter), fused_modconv=fused_modconv, styles=next(s_iter), **layer_kwargs)
        elif self.architecture == 'resnet':
            y = self.skip(x, gain=np.sqrt(0.5))
            x = self.conv0(x, next(w_iter), fused_modconv=fused_modconv, styles=next(s_iter), **layer_kwargs)
            x = self.conv1(x, next(w_iter), fused_modconv=fused_modconv, gain=np.sqrt(0.5), styles=next(s_iter),
                           **layer_kwargs)
            x = y.add_(x)
        else:
            x = self.conv0(x, next(w_iter), fused_modconv=fused_modconv, styles=next(s_iter), **layer_kwargs)
            x = self.conv1(x, next(w_iter), fused_modconv=fused_modconv, styles=next(s_iter), **layer_kwargs)
        if img is not None:
            misc.assert_shape(img, [None, self.img_channels, self.resolution // 2, self.resolution // 2])
            img = upfirdn2d.upsample2d(img, self.resample_filter)
        if self.is_last or self.architecture == 'skip':
            if self.is_last:
                y = self.torgb(x, next(w_iter), fused_modconv=fused_modconv, styles=next(s_iter))
            else:     # x feeds the next block too
                x, y = self.torgb.forward_tap(x, next(w_iter), fused_modconv=fused_modconv, styles=next(s_iter))
            y = y.to(dtype=torch.float32, memory_format=torch.contiguous_format)
            img = img.add_(y) if img is not None else y
        assert x.dtype == dtype
        assert img is None or img.dtype == torch.float32
        return x, img

    def extra_repr(self):
        return f'resolution={self.resolution:d}, architecture={self.architecture:s}'


@persistence.persistent_class
class SynthesisNetwork(torch.nn.Module):
    """:466-522"""

    def __init__(self, w_dim, img_resolution, img_channels, channel_base=32768, channel_max=512, num_fp16_res=4,
                 **block_kwargs):
        assert img_resolution >= 4 and img_resolution & (img_resolution - 1) == 0
        super().__init__()
        self.w_dim, self.img_resolution, self.img_channels = w_dim, img_resolution, img_channels
        self.img_resolution_log2 = int(np.log2(img_resolution))
        self.num_fp16_res = num_fp16_res
        self.block_resolutions = [2 ** i for i in range(2, self.img_resolution_log2 + 1)]
        channels = {r: min(channel_base // r, channel_max) for r in self.block_resolutions}
        fp16_resolution = max(2 ** (self.img_resolution_log2 + 1 - num_fp16_res), 8)
        self.num_ws = 0
        for r in self.block_resolutions:
            block = SynthesisBlock(channels[r // 2] if r > 4 else 0, channels[r], w_dim=w_dim, resolution=r,
                                   img_channels=img_channels, is_last=(r == img_resolution),
                                   use_fp16=(r >= fp16_resolution), **block_kwargs)
            self.num_ws += block.num_conv
            if r == img_resolution:
                self.num_ws += block.num_torgb
            setattr(self, f'b{r}', block)

    def forward(self, ws, **block_kwargs):
        misc.assert_shape(ws, [None, self.num_ws, self.w_dim])
        ws = ws.to(torch.float32)
        x = img = None
        styles = None
        if grouped_affine and ws.is_cuda:
            plan, w_idx = [], 0
            for r in self.block_resolutions:
                block = getattr(self, f'b{r}')
                plan += [(a, w_idx + k, g) for a, k, g in block.style_layers()]
                w_idx += block.num_conv
            styles = iter(grouped_styles(ws, plan))
        w_idx = 0
        for r in self.block_resolutions:
            block = getattr(self, f'b{r}')
            cur = ws.narrow(1, w_idx, block.num_conv + block.num_torgb)
            w_idx += block.num_conv
            bs = [next(styles) for _ in block.style_layers()] if styles is not None else None
            x, img = block(x, img, cur, styles=bs, **block_kwargs)
        return img

    def extra_repr(self):
        return (f'w_dim={self.w_dim:d}, num_ws={self.num_ws:d}, img_resolution={self.img_resolution:d}, '
                f'img_channels={self.img_channels:d}, num_fp16_res={self.num_fp16_res:d}')


@persistence.persistent_class
class Generator(torch.nn.Module):
    """:526-550"""

    def __init__(self, z_dim, c_dim, w_dim, img_resolution, img_channels, mapping_kwargs={}, **synthesis_kwargs):
        super().__init__()
        self.z_dim, self.c_dim, self.w_dim = z_dim, c_dim, w_dim
        self.img_resolution, self.img_channels = img_resolution, img_channels
        self.synthesis = SynthesisNetwork(w_dim=w_dim, img_resolution=img_resolution, img_channels=img_channels,
                                          **synthesis_kwargs)
        self.num_ws = self.synthesis.num_ws
        self.mapping = MappingNetwork(z_dim=z_dim, c_dim=c_dim, w_dim=w_dim, num_ws=self.num_ws, **mapping_kwargs)

    def forward(self, z, c, truncation_psi=1, truncation_cutoff=None, update_emas=False, **synthesis_kwargs):
        ws = self.mapping(z, c, truncation_psi=truncation_psi, truncation_cutoff=truncation_cutoff,
                          update_emas=update_emas)
        return self.synthesis(ws, update_emas=update_emas, **synthesis_kwargs)


@persistence.persistent_class
class DiscriminatorBlock(torch.nn.Module):
    """:554-639"""

    def __init__(self, in_channels, tmp_channels, out_channels, resolution, img_channels, first_layer_idx,
                 architecture='resnet', activation='lrelu', resample_filter=[1, 3, 3, 1], conv_clamp=None,
                 use_fp16=False, fp16_channels_last=False, freeze_layers=0, fp16_dtype=torch.float16):
        assert in_channels in [0, tmp_channels]
        assert architecture in ['orig', 'skip', 'resnet']
        super().__init__()
        self.in_channels, self.resolution, self.img_channels = in_channels, resolution, img_channels
        self.first_layer_idx, self.architecture = first_layer_idx, architecture
        self.use_fp16, self.fp16_dtype = use_fp16, fp16_dtype
        self.channels_last = True
        self.register_buffer('resample_filter', upfirdn2d.setup_filter(resample_filter))
        self.num_layers = 0

        def next_trainable():
            layer_idx = self.first_layer_idx + self.num_layers
            self.num_layers += 1
            return layer_idx >= freeze_layers

        if in_channels == 0 or architecture == 'skip':
            self.fromrgb = Conv2dLayer(img_channels, tmp_channels, kernel_size=1, activation=activation,
                                       trainable=next_trainable(), conv_clamp=conv_clamp)
        self.conv0 = Conv2dLayer(tmp_channels, tmp_channels, kernel_size=3, activation=activation,
                                 trainable=next_trainable(), conv_clamp=conv_clamp)
        self.conv1 = Conv2dLayer(tmp_channels, out_channels, kernel_size=3, activation=activation, down=2,
                                 trainable=next_trainable(), resample_filter=resample_filter, conv_clamp=conv_clamp)
        if architecture == 'resnet':
            self.skip = Conv2dLayer(tmp_channels, out_channels, kernel_size=1, bias=False, down=2,
                                    trainable=next_trainable(), resample_filter=resample_filter)

    def forward(self, x, img, force_fp32=False):
        dtype = self.fp16_dtype if self.use_fp16 and not force_fp32 else torch.float32
        if x is not None:
            misc.assert_shape(x, [None, self.in_channels, self.resolution, self.resolution])
            x = x.to(dtype=dtype, memory_format=_CL)
        if self.in_channels == 0 or self.architecture == 'skip':
            misc.assert_shape(img, [None, self.img_channels, self.resolution, self.resolution])
            img = img.to(dtype=dtype, memory_format=_CL)
            y = self.fromrgb(img)
            x = x + y if x is not None else y
            img = upfirdn2d.downsample2d(img, self.resample_filter) if self.architecture == 'skip' else None
        if self.architecture == 'resnet':
            sk = self.skip
            if sk.down > 1 and sk.weight.shape[2] == 1 and upfirdn2d.fork_fir_ok(x, sk.resample_filter):
                # the skip's FIR taken off x with the two branches' gradient add fused into its backward
                pad = conv2d_resample._frame_padding(sk.padding, sk.resample_filter, 1, sk.down)
                x, xd = upfirdn2d.fork_fir(x, sk.resample_filter, sk.down, pad)
                y = sk(xd, gain=np.sqrt(0.5), prefiltered=True)
            else:
                y = self.skip(x, gain=np.sqrt(0.5))
            x = self.conv0(x)
            x = self.conv1(x, gain=np.sqrt(0.5), residual=y)   # y + conv1(x), the add fused into conv1
        else:
            x = self.conv0(x)
            x = self.conv1(x)
        assert x.dtype == dtype
        return x, img

    def extra_repr(self):
        return f'resolution={self.resolution:d}, architecture={self.architecture:s}'


@persistence.persistent_class
class MinibatchStdLayer(torch.nn.Module):
    """:643-668"""

    def __init__(self, group_size, num_channels=1):
        super().__init__()
        self.group_size, self.num_channels = group_size, num_channels
        self.segments = None    # sizes of independent sub-batches (batched D passes, see loss.py), or None

    def forward(self, x):
        seg = getattr(self, 'segments', None)
        if seg is not None and len(seg) > 1:
            # the statistics are taken within each sub-batch, as separate D passes would
            return torch.cat([self._forward(part) for part in x.split(list(seg))])
        return self._forward(x)

    def _forward(self, x):
        N, C, H, W = x.shape
        G = min(self.group_size, N) if self.group_size is not None else N
        F = self.num_channels
        c = C // F
        y = x.reshape(G, -1, F, c, H, W)
        y = y - y.mean(dim=0)
        y = y.square().mean(dim=0)
        y = (y + 1e-8).sqrt()
        y = y.mean(dim=[2, 3, 4])
        y = y.reshape(-1, F, 1, 1).repeat(G, 1, H, W)
        return torch.cat([x, y], dim=1)

    def extra_repr(self):
        return f'group_size={self.group_size}, num_channels={self.num_channels:d}'


@persistence.persistent_class
class DiscriminatorEpilogue(torch.nn.Module):
    """:672-729 (runs in float32, like the reference)."""

    def __init__(self, in_channels, cmap_dim, resolution, img_channels, architecture='resnet', mbstd_group_size=4,
                 mbstd_num_channels=1, activation='lrelu', conv_clamp=None):
        assert architecture in ['orig', 'skip', 'resnet']
        super().__init__()
        self.in_channels, self.cmap_dim, self.resolution = in_channels, cmap_dim, resolution
        self.img_channels, self.architecture = img_channels, architecture
        if architecture == 'skip':
            self.fromrgb = Conv2dLayer(img_channels, in_channels, kernel_size=1, activation=activation)
        self.mbstd = MinibatchStdLayer(group_size=mbstd_group_size, num_channels=mbstd_num_channels) \
            if mbstd_num_channels > 0 else None
        self.conv = Conv2dLayer(in_channels + mbstd_num_channels, in_channels, kernel_size=3, activation=activation,
                                conv_clamp=conv_clamp)
        self.fc = FullyConnectedLayer(in_channels * (resolution ** 2), in_channels, activation=activation)
        self.out = FullyConnectedLayer(in_channels, 1 if cmap_dim == 0 else cmap_dim)

    def forward(self, x, img, cmap, force_fp32=False):
        misc.assert_shape(x, [None, self.in_channels, self.resolution, self.resolution])
        x = x.to(dtype=torch.float32, memory_format=torch.contiguous_format)
        if self.architecture == 'skip':
            img = img.to(dtype=torch.float32, memory_format=torch.contiguous_format)
            x = x + self.fromrgb(img)
        if self.mbstd is not None:
            x = self.mbstd(x)
        x = self.conv(x)
        x = self.fc(x.contiguous().flatten(1))
        x = self.out(x)
        if self.cmap_dim > 0:
            misc.assert_shape(cmap, [None, self.cmap_dim])
            x = (x * cmap).sum(dim=1, keepdim=True) * (1 / np.sqrt(self.cmap_dim))
        assert x.dtype == torch.float32
        return x

    def extra_repr(self):
        return f'resolution={self.resolution:d}, architecture={self.architecture:s}'


@persistence.persistent_class
class Discriminator(torch.nn.Module):
    """:733-792"""

    def __init__(self, c_dim, img_resolution, img_channels, architecture='resnet', channel_base=32768,
                 channel_max=512, num_fp16_res=4, conv_clamp=256, cmap_dim=None, block_kwargs={}, mapping_kwargs={},
                 epilogue_kwargs={}):
        super().__init__()
        self.c_dim, self.img_resolution, self.img_channels = c_dim, img_resolution, img_channels
        self.img_resolution_log2 = int(np.log2(img_resolution))
        self.block_resolutions = [2 ** i for i in range(self.img_resolution_log2, 2, -1)]
        channels = {r: min(channel_base // r, channel_max) for r in self.block_resolutions + [4]}
        fp16_resolution = max(2 ** (self.img_resolution_log2 + 1 - num_fp16_res), 8)
        if cmap_dim is None:
            cmap_dim = channels[4]
        if c_dim == 0:
            cmap_dim = 0
        common = dict(img_channels=img_channels, architecture=architecture, conv_clamp=conv_clamp)
        layer_idx = 0
        for r in self.block_resolutions:
            block = DiscriminatorBlock(channels[r] if r < img_resolution else 0, channels[r], channels[r // 2],
                                       resolution=r, first_layer_idx=layer_idx, use_fp16=(r >= fp16_resolution),
                                       **block_kwargs, **common)
            setattr(self, f'b{r}', block)
            layer_idx += block.num_layers
        if c_dim > 0:
            self.mapping = MappingNetwork(z_dim=0, c_dim=c_dim, w_dim=cmap_dim, num_ws=None, w_avg_beta=None,
                                          **mapping_kwargs)
        self.b4 = DiscriminatorEpilogue(channels[4], cmap_dim=cmap_dim, resolution=4, **epilogue_kwargs, **common)

    def forward(self, img, c, update_emas=False, **block_kwargs):
        x = None
        for r in self.block_resolutions:
            x, img = getattr(self, f'b{r}')(x, img, **block_kwargs)
        cmap = self.mapping(None, c) if self.c_dim > 0 else None
        return self.b4(x, img, cmap)

    def extra_repr(self):
        return f'c_dim={self.c_dim:d}, img_resolution={self.img_resolution:d}, img_channels={self.img_channels:d}'
