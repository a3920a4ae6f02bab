"""ORACLE -- CPU restatement of the reference StyleGAN2-ADA training path (test infrastructure).

This file is the parity checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.  It restates,
in plain PyTorch on the CPU (fp32/fp64), the algorithm of the reference
(ltronchin/Gan-track @ v0, vendored NVIDIA StyleGAN3 code under src/models/stylegan3 = ``SG3/``),
function by function, each citing the reference ``file:line`` it follows.

Pinning: ``tests/test_oracle_golden.py`` checks every function here against golden vectors
produced by importing the reference itself on CPU (``tests/golden/make_golden.py``):
upfirdn2d, bias_act (1st/2nd order), modulated_conv2d, Conv2dLayer/conv2d_resample,
AugmentPipe (debug-percentile and RNG-taped paths), G/D forward and one full training
iteration (Gmain/Greg/Dmain/Dreg + lazy-reg Adam + EMA).

Parameter / buffer names equal the reference's so state dicts interchange.
"""
import copy

import numpy as np
import torch
import torch.nn.functional as F

# The oracle's real type.  float32 is the reference's CPU arithmetic; tests/golden/make_golden.py sets
# float64 to evaluate the exact (rounding-free) answer the fp32 results are judged against.
REAL = torch.float32

# 16-bit emulation (None, torch.float16 or torch.bfloat16).  The reference on a GPU runs its top num_fp16_res
# blocks in float16 (networks_stylegan2.py:419-420, :607-608): every op of such a block produces a 16-bit tensor
# -- computed in f32 by the kernel (cuDNN / the plugins / torch's opmath) and rounded once -- and autograd
# produces each of those tensors' gradients in 16 bits too.  With EMU16 set, the blocks flagged use_fp16 round
# every such tensor to EMU16 (forward value and incoming gradient, _Round16) at exactly those points, while the
# arithmetic in between stays REAL: the oracle then evaluates the reference's 16-bit GPU iteration (to its
# f32-versus-REAL accumulation difference), the yardstick the product's 16-bit results are held to.
EMU16 = None
# EMU16 = torch.float32 emulates an f32 evaluation instead: EVERY block rounds at those points (num_fp16_res plays
# no part), and with EMU_JITTER (a numpy Generator: torch draws would enter the RNG tapes that replay the
# reference's draws) each value is first nudged by a random fraction of an f32 ulp
# (|u| < 2^-24 relative) -- independent samples of the rounding an f32 implementation of the same algorithm
# makes, to measure how far f32 rounding alone can move a result (tests/golden/make_golden.py `emu32:`).
EMU_JITTER = None


class _Round16(torch.autograd.Function):
    """y = round_to_16bit(x); dL/dx = round_to_16bit(dL/dy) (the gradient of a 16-bit tensor is a 16-bit tensor);
    differentiable again for the double backward."""

    @staticmethod
    def forward(ctx, x, dt):
        ctx.dt = dt
        if dt == torch.float32 and EMU_JITTER is not None:
            u = torch.from_numpy(EMU_JITTER.uniform(-1.0, 1.0, tuple(x.shape))).to(x.dtype)
            x = x * (1 + u * 2.0 ** -24)
        return x.to(dt).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return _Round16.apply(g, ctx.dt), None


def _q(x, on):
    """Round to the emulated 16-bit type inside a use_fp16 block (identity otherwise)."""
    if not on or EMU16 is None or x is None:
        return x
    return _Round16.apply(x, EMU16)

# =============================================================================================
# upfirdn2d  (SG3/torch_utils/ops/upfirdn2d.py)
# =============================================================================================


def _pair(v):
    if isinstance(v, int):
        return v, v
    a, b = v
    return int(a), int(b)


def _pad4(p):
    if isinstance(p, int):
        return p, p, p, p
    if len(p) == 2:
        return p[0], p[0], p[1], p[1]
    return tuple(int(v) for v in p)


def filter_size(f):
    """SG3 upfirdn2d.py:55-66 -> (fw, fh)."""
    if f is None:
        return 1, 1
    return int(f.shape[-1]), int(f.shape[0])


def setup_filter(f, normalize=True, flip_filter=False, gain=1, separable=None):
    """SG3 upfirdn2d.py:70-114."""
    f = torch.as_tensor(1 if f is None else f, dtype=REAL)
    if f.ndim == 0:
        f = f.reshape(1)
    if separable is None:
        separable = (f.ndim == 1 and f.numel() >= 8)
    if f.ndim == 1 and not separable:
        f = torch.outer(f, f)
    if normalize:
        f = f / f.sum()
    if flip_filter:
        f = f.flip(list(range(f.ndim)))
    return f * (gain ** (f.ndim / 2))


def upfirdn2d(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1):
    """Zero-insert upsample, pad/crop, FIR, decimate.  SG3 upfirdn2d.py:166-211."""
    return _upfirdn2d_(x, f, up, down, padding, flip_filter, gain)


def _upfirdn2d_(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1):
    if f is None:
        f = torch.ones([1, 1], dtype=REAL)
    n, c, h, w = x.shape
    ux, uy = _pair(up)
    dx, dy = _pair(down)
    px0, px1, py0, py1 = _pad4(padding)
    # 1. upsample by zero insertion
    z = x.new_zeros([n, c, h, uy, w, ux])
    z[:, :, :, 0, :, 0] = x
    z = z.reshape(n, c, h * uy, w * ux)
    # 2. pad (positive) then crop (negative)
    z = F.pad(z, [max(px0, 0), max(px1, 0), max(py0, 0), max(py1, 0)])
    z = z[:, :, max(-py0, 0): z.shape[2] - max(-py1, 0), max(-px0, 0): z.shape[3] - max(-px1, 0)]
    # 3. FIR (true convolution unless flip_filter)
    f = (f * (gain ** (f.ndim / 2))).to(x.dtype)
    if not flip_filter:
        f = f.flip(list(range(f.ndim)))
    if f.ndim == 2:
        z = F.conv2d(z, f[None, None].expand(c, 1, *f.shape), groups=c)
    else:
        z = F.conv2d(z, f[None, None, None, :].expand(c, 1, 1, f.shape[0]), groups=c)
        z = F.conv2d(z, f[None, None, :, None].expand(c, 1, f.shape[0], 1), groups=c)
    # 4. decimate
    return z[:, :, ::dy, ::dx]


def upsample2d(x, f, up=2, padding=0, flip_filter=False, gain=1):
    """SG3 upfirdn2d.py:313-348."""
    ux, uy = _pair(up)
    px0, px1, py0, py1 = _pad4(padding)
    fw, fh = filter_size(f)
    p = [px0 + (fw + ux - 1) // 2, px1 + (fw - ux) // 2, py0 + (fh + uy - 1) // 2, py1 + (fh - uy) // 2]
    return upfirdn2d(x, f, up=up, padding=p, flip_filter=flip_filter, gain=gain * ux * uy)


def downsample2d(x, f, down=2, padding=0, flip_filter=False, gain=1):
    """SG3 upfirdn2d.py:352-387."""
    dx, dy = _pair(down)
    px0, px1, py0, py1 = _pad4(padding)
    fw, fh = filter_size(f)
    p = [px0 + (fw - dx + 1) // 2, px1 + (fw - dx) // 2, py0 + (fh - dy + 1) // 2, py1 + (fh - dy) // 2]
    return upfirdn2d(x, f, down=down, padding=p, flip_filter=flip_filter, gain=gain)


def filter2d(x, f, padding=0, flip_filter=False, gain=1):
    """SG3 upfirdn2d.py:277-309."""
    px0, px1, py0, py1 = _pad4(padding)
    fw, fh = filter_size(f)
    p = [px0 + fw // 2, px1 + (fw - 1) // 2, py0 + fh // 2, py1 + (fh - 1) // 2]
    return upfirdn2d(x, f, padding=p, flip_filter=flip_filter, gain=gain)


# =============================================================================================
# bias_act  (SG3/torch_utils/ops/bias_act.py:21-120)
# =============================================================================================

# name -> (function, default alpha, default gain, reference cuda_idx, has 2nd grad)
ACTIVATIONS = {
    'linear': (lambda x, a: x, 0.0, 1.0, 1, False),
    'relu': (lambda x, a: F.relu(x), 0.0, float(np.sqrt(2)), 2, False),
    'lrelu': (lambda x, a: F.leaky_relu(x, a), 0.2, float(np.sqrt(2)), 3, False),
    'tanh': (lambda x, a: torch.tanh(x), 0.0, 1.0, 4, True),
    'sigmoid': (lambda x, a: torch.sigmoid(x), 0.0, 1.0, 5, True),
    'elu': (lambda x, a: F.elu(x), 0.0, 1.0, 6, True),
    'selu': (lambda x, a: F.selu(x), 0.0, 1.0, 7, True),
    'softplus': (lambda x, a: F.softplus(x), 0.0, 1.0, 8, True),
    'swish': (lambda x, a: torch.sigmoid(x) * x, 0.0, float(np.sqrt(2)), 9, True),
}


def bias_act(x, b=None, dim=1, act='linear', alpha=None, gain=None, clamp=None):
    fn, da, dg, _, _ = ACTIVATIONS[act]
    alpha = float(da if alpha is None else alpha)
    gain = float(dg if gain is None else gain)
    if b is not None:
        shape = [1] * x.ndim
        shape[dim] = -1
        x = x + b.reshape(shape)
    x = fn(x, alpha)
    if gain != 1:
        x = x * gain
    if clamp is not None and clamp >= 0:
        x = x.clamp(-clamp, clamp)
    return x


# =============================================================================================
# grid_sample with double backward  (SG3/torch_utils/ops/grid_sample_gradfix.py:28-83)
# =============================================================================================


class _GridSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inp, grid):
        ctx.save_for_backward(inp, grid)
        return F.grid_sample(inp, grid, mode='bilinear', padding_mode='zeros', align_corners=False)

    @staticmethod
    def backward(ctx, gout):
        inp, grid = ctx.saved_tensors
        return _GridSampleBwd.apply(gout, inp, grid), None


class _GridSampleBwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gout, inp, grid):
        gi, _ = torch.ops.aten.grid_sampler_2d_backward(gout, inp, grid, 0, 0, False, [True, False])
        ctx.save_for_backward(grid)
        return gi

    @staticmethod
    def backward(ctx, ggi):
        grid, = ctx.saved_tensors
        return _GridSample.apply(ggi, grid), None, None


def grid_sample(inp, grid):
    return _GridSample.apply(inp, grid)


# =============================================================================================
# conv2d_resample  (SG3/torch_utils/ops/conv2d_resample.py:21-141)
# =============================================================================================


def _conv_(x, w, stride=1, padding=0, groups=1, transpose=False, flip_weight=True):
    if not flip_weight and (w.shape[2] > 1 or w.shape[3] > 1):
        w = w.flip([2, 3])
    if transpose:
        return F.conv_transpose2d(x, w, stride=stride, padding=padding, groups=groups)
    return F.conv2d(x, w, stride=stride, padding=padding, groups=groups)


def conv2d_resample(x, w, f=None, up=1, down=1, padding=0, groups=1, flip_weight=True, flip_filter=False, q16=False):
    """q16: every intermediate is a 16-bit tensor (EMU16), as the reference's fp16 blocks run it."""
    if q16 and EMU16 is not None:
        def _conv(*a, **k):
            return _q(_conv_(*a, **k), True)

        def upfirdn2d(*a, **k):
            return _q(_upfirdn2d_(*a, **k), True)
    else:
        _conv, upfirdn2d = _conv_, _upfirdn2d_
    oc, icg, kh, kw = w.shape
    fw, fh = filter_size(f)
    px0, px1, py0, py1 = _pad4(padding)
    if up > 1:
        px0 += (fw + up - 1) // 2
        px1 += (fw - up) // 2
        py0 += (fh + up - 1) // 2
        py1 += (fh - up) // 2
    if down > 1:
        px0 += (fw - down + 1) // 2
        px1 += (fw - down) // 2
        py0 += (fh - down + 1) // 2
        py1 += (fh - down) // 2
    if kw == 1 and kh == 1 and down > 1 and up == 1:                      # :94-97
        x = upfirdn2d(x, f, down=down, padding=[px0, px1, py0, py1], flip_filter=flip_filter)
        return _conv(x, w, groups=groups, flip_weight=flip_weight)
    if kw == 1 and kh == 1 and up > 1 and down == 1:                      # :100-103
        x = _conv(x, w, groups=groups, flip_weight=flip_weight)
        return upfirdn2d(x, f, up=up, padding=[px0, px1, py0, py1], gain=up ** 2, flip_filter=flip_filter)
    if down > 1 and up == 1:                                              # :106-109
        x = upfirdn2d(x, f, padding=[px0, px1, py0, py1], flip_filter=flip_filter)
        return _conv(x, w, stride=down, groups=groups, flip_weight=flip_weight)
    if up > 1:                                                            # :112-129
        if groups == 1:
            w = w.transpose(0, 1)
        else:
            w = w.reshape(groups, oc // groups, icg, kh, kw).transpose(1, 2).reshape(groups * icg, oc // groups, kh, kw)
        px0 -= kw - 1
        px1 -= kw - up
        py0 -= kh - 1
        py1 -= kh - up
        pxt = max(min(-px0, -px1), 0)
        pyt = max(min(-py0, -py1), 0)
        x = _conv(x, w, stride=up, padding=[pyt, pxt], groups=groups, transpose=True, flip_weight=not flip_weight)
        x = upfirdn2d(x, f, padding=[px0 + pxt, px1 + pxt, py0 + pyt, py1 + pyt], gain=up ** 2, flip_filter=flip_filter)
        if down > 1:
            x = upfirdn2d(x, f, down=down, flip_filter=flip_filter)
        return x
    if up == 1 and down == 1 and px0 == px1 and py0 == py1 and px0 >= 0 and py0 >= 0:   # :132-134
        return _conv(x, w, padding=[py0, px0], groups=groups, flip_weight=flip_weight)
    x = upfirdn2d(x, f if up > 1 else None, up=up, padding=[px0, px1, py0, py1], gain=up ** 2, flip_filter=flip_filter)
    x = _conv(x, w, groups=groups, flip_weight=flip_weight)
    if down > 1:
        x = upfirdn2d(x, f, down=down, flip_filter=flip_filter)
    return x


# =============================================================================================
# networks  (SG3/training/networks_stylegan2.py)
# =============================================================================================


def normalize_2nd_moment(x, dim=1, eps=1e-8):
    """:26-27"""
    return x * (x.square().mean(dim=dim, keepdim=True) + eps).rsqrt()


def modulated_conv2d(x, weight, styles, noise=None, up=1, down=1, padding=0, resample_filter=None,
                     demodulate=True, flip_weight=True, fused_modconv=True, q16=False):
    """:32-89 (the fp16 pre-normalisation :52-54 applies only to fp16 inputs: EMU16 float16 in a q16 block)."""
    n = x.shape[0]
    oc, ic, kh, kw = weight.shape
    q = q16 and EMU16 is not None
    if q and EMU16 == torch.float16 and demodulate:                     # :52-54
        weight = weight * (1 / np.sqrt(ic * kh * kw) / weight.norm(float('inf'), dim=[1, 2, 3], keepdim=True))
        styles = styles / styles.norm(float('inf'), dim=1, keepdim=True)
    w = dcoefs = None
    if demodulate or fused_modconv:
        w = weight.unsqueeze(0) * styles.reshape(n, 1, -1, 1, 1)
    if demodulate:
        dcoefs = (w.square().sum(dim=[2, 3, 4]) + 1e-8).rsqrt()
    if demodulate and fused_modconv:
        w = w * dcoefs.reshape(n, -1, 1, 1, 1)
    if not fused_modconv:
        x = _q(x * _q(styles, q).reshape(n, -1, 1, 1), q)                  # :69-70, weight.to(x.dtype)
        x = conv2d_resample(x, _q(weight, q), f=resample_filter, up=up, down=down, padding=padding,
                            flip_weight=flip_weight, q16=q)
        if demodulate and noise is not None:                                # fma.fma: one rounding
            return _q(torch.addcmul(_q(noise, q), x, _q(dcoefs, q).reshape(n, -1, 1, 1)), q)
        if demodulate:
            return _q(x * _q(dcoefs, q).reshape(n, -1, 1, 1), q)
        if noise is not None:
            return _q(x + _q(noise, q), q)
        return x
    x = x.reshape(1, -1, *x.shape[2:])
    w = w.reshape(-1, ic, kh, kw)
    x = conv2d_resample(x, w, f=resample_filter, up=up, down=down, padding=padding, groups=n, flip_weight=flip_weight)
    x = x.reshape(n, -1, *x.shape[2:])
    if noise is not None:
        x = x + noise
    return x


class FullyConnectedLayer(torch.nn.Module):
    """:94-125"""

    def __init__(self, in_features, out_features, bias=True, activation='linear', lr_multiplier=1, bias_init=0):
        super().__init__()
        self.activation = activation
        self.weight = torch.nn.Parameter(torch.randn([out_features, in_features]) / lr_multiplier)
        self.bias = torch.nn.Parameter(torch.full([out_features], float(np.float32(bias_init)), dtype=REAL)) if bias else None
        self.weight_gain = lr_multiplier / np.sqrt(in_features)
        self.bias_gain = lr_multiplier

    def forward(self, x):
        w = self.weight * self.weight_gain
        b = self.bias
        if b is not None and self.bias_gain != 1:
            b = b * self.bias_gain
        if self.activation == 'linear' and b is not None:
            return torch.addmm(b.unsqueeze(0), x, w.t())
        return bias_act(x.matmul(w.t()), b, act=self.activation)


class Conv2dLayer(torch.nn.Module):
    """:133-181"""

    def __init__(self, in_channels, out_channels, kernel_size, bias=True, activation='linear', up=1, down=1,
                 resample_filter=(1, 3, 3, 1), conv_clamp=None, channels_last=False, trainable=True):
        super().__init__()
        self.activation = activation
        self.up, self.down = up, down
        self.conv_clamp = conv_clamp
        self.register_buffer('resample_filter', setup_filter(list(resample_filter)))
        self.padding = kernel_size // 2
        self.weight_gain = 1 / np.sqrt(in_channels * kernel_size ** 2)
        self.act_gain = ACTIVATIONS[activation][2]
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

    def forward(self, x, gain=1, q16=False):
        w = self.weight * self.weight_gain
        x = conv2d_resample(x, _q(w, q16), f=self.resample_filter, up=self.up, down=self.down, padding=self.padding,
                            flip_weight=(self.up == 1), q16=q16)
        clamp = self.conv_clamp * gain if self.conv_clamp is not None else None
        return _q(bias_act(x, _q(self.bias, q16), act=self.activation, gain=self.act_gain * gain, clamp=clamp), q16)


class MappingNetwork(torch.nn.Module):
    """:191-266"""

    def __init__(self, z_dim, c_dim, w_dim, num_ws, num_layers=8, embed_features=None, layer_features=None,
                 activation='lrelu', lr_multiplier=0.01, w_avg_beta=0.998):
        super().__init__()
        self.z_dim, self.c_dim, self.w_dim, self.num_ws = z_dim, c_dim, w_dim, num_ws
        self.num_layers, self.w_avg_beta = num_layers, w_avg_beta
        embed_features = w_dim if embed_features is None else embed_features
        if c_dim == 0:
            embed_features = 0
        layer_features = w_dim if layer_features is None else layer_features
        feats = [z_dim + embed_features] + [layer_features] * (num_layers - 1) + [w_dim]
        if c_dim > 0:
            self.embed = FullyConnectedLayer(c_dim, embed_features)
        for i in range(num_layers):
            setattr(self, f'fc{i}', FullyConnectedLayer(feats[i], feats[i + 1], activation=activation,
                                                        lr_multiplier=lr_multiplier))
        if num_ws is not None and w_avg_beta is not None:
            self.register_buffer('w_avg', torch.zeros([w_dim]))

    def forward(self, z, c, truncation_psi=1, truncation_cutoff=None, update_emas=False):
        x = None
        if self.z_dim > 0:
            x = normalize_2nd_moment(z.to(REAL))
        if self.c_dim > 0:
            y = normalize_2nd_moment(self.embed(c.to(REAL)))
            x = torch.cat([x, y], dim=1) if x is not None else y
        for i in range(self.num_layers):
            x = getattr(self, f'fc{i}')(x)
        if update_emas and self.w_avg_beta is not None:
            self.w_avg.copy_(x.detach().mean(dim=0).lerp(self.w_avg, self.w_avg_beta))
        if self.num_ws is not None:
            x = x.unsqueeze(1).repeat([1, self.num_ws, 1])
        if truncation_psi != 1:
            if self.num_ws is None or truncation_cutoff is None:
                x = self.w_avg.lerp(x, truncation_psi)
            else:
                x[:, :truncation_cutoff] = self.w_avg.lerp(x[:, :truncation_cutoff], truncation_psi)
        return x


class SynthesisLayer(torch.nn.Module):
    """:273-333"""

    def __init__(self, in_channels, out_channels, w_dim, resolution, kernel_size=3, up=1, use_noise=True,
                 activation='lrelu', resample_filter=(1, 3, 3, 1), conv_clamp=None, channels_last=False):
        super().__init__()
        self.resolution, self.up, self.use_noise = resolution, up, use_noise
        self.activation, self.conv_clamp = activation, conv_clamp
        self.register_buffer('resample_filter', setup_filter(list(resample_filter)))
        self.padding = kernel_size // 2
        self.act_gain = ACTIVATIONS[activation][2]
        self.affine = FullyConnectedLayer(w_dim, in_channels, bias_init=1)
        self.weight = torch.nn.Parameter(torch.randn([out_channels, in_channels, kernel_size, kernel_size]))
        if use_noise:
            self.register_buffer('noise_const', torch.randn([resolution, resolution]))
            self.noise_strength = torch.nn.Parameter(torch.zeros([]))
        self.bias = torch.nn.Parameter(torch.zeros([out_channels]))

    def forward(self, x, w, noise_mode='random', fused_modconv=True, gain=1, q16=False):
        styles = self.affine(w)
        noise = None
        if self.use_noise and noise_mode == 'random':
            noise = torch.randn([x.shape[0], 1, self.resolution, self.resolution], device=x.device) * self.noise_strength
        if self.use_noise and noise_mode == 'const':
            noise = self.noise_const * self.noise_strength
        x = modulated_conv2d(x, self.weight, styles, noise=noise, up=self.up, padding=self.padding,
                             resample_filter=self.resample_filter, flip_weight=(self.up == 1),
                             fused_modconv=fused_modconv, q16=q16)
        clamp = self.conv_clamp * gain if self.conv_clamp is not None else None
        return _q(bias_act(x, _q(self.bias, q16), act=self.activation, gain=self.act_gain * gain, clamp=clamp), q16)


class ToRGBLayer(torch.nn.Module):
    """:337-358"""

    def __init__(self, in_channels, out_channels, w_dim, kernel_size=1, conv_clamp=None, channels_last=False):
        super().__init__()
        self.conv_clamp = conv_clamp
        self.affine = FullyConnectedLayer(w_dim, in_channels, bias_init=1)
        self.weight = torch.nn.Parameter(torch.randn([out_channels, in_channels, kernel_size, kernel_size]))
        self.bias = torch.nn.Parameter(torch.zeros([out_channels]))
        self.weight_gain = 1 / np.sqrt(in_channels * kernel_size ** 2)

    def forward(self, x, w, fused_modconv=True, q16=False):
        styles = self.affine(w) * self.weight_gain
        x = modulated_conv2d(x, self.weight, styles, demodulate=False, fused_modconv=fused_modconv, q16=q16)
        return _q(bias_act(x, _q(self.bias, q16), clamp=self.conv_clamp), q16)


class SynthesisBlock(torch.nn.Module):
    """:362-462 (fp32 / contiguous: the reference forces fp32 off-CUDA, :419-420)."""

    def __init__(self, in_channels, out_channels, w_dim, resolution, img_channels, is_last, architecture='skip',
                 resample_filter=(1, 3, 3, 1), conv_clamp=256, use_fp16=False, fp16_channels_last=False,
                 fused_modconv_default=True, **layer_kwargs):
        super().__init__()
        self.in_channels, self.resolution, self.img_channels = in_channels, resolution, img_channels
        self.is_last, self.architecture, self.use_fp16 = is_last, architecture, use_fp16
        self.fused_modconv_default = fused_modconv_default
        self.register_buffer('resample_filter', setup_filter(list(resample_filter)))
        self.num_conv = self.num_torgb = 0
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

    def forward(self, x, img, ws, force_fp32=False, fused_modconv=None, update_emas=False, **layer_kwargs):
        w_iter = iter(ws.unbind(dim=1))
        if fused_modconv is None:
            fused_modconv = self.fused_modconv_default
        if fused_modconv == 'inference_only':
            fused_modconv = not self.training
        q = (self.use_fp16 or EMU16 == torch.float32) and EMU16 is not None and not force_fp32   # :419-420
        if self.in_channels == 0:
            x = _q(self.const, q).unsqueeze(0).repeat([ws.shape[0], 1, 1, 1])
            x = self.conv1(x, next(w_iter), fused_modconv=fused_modconv, q16=q, **layer_kwargs)
        elif self.architecture == 'resnet':
            x = _q(x, q)
            y = self.skip(x, gain=np.sqrt(0.5), q16=q)
            x = self.conv0(x, next(w_iter), fused_modconv=fused_modconv, q16=q, **layer_kwargs)
            x = self.conv1(x, next(w_iter), fused_modconv=fused_modconv, gain=np.sqrt(0.5), q16=q, **layer_kwargs)
            x = _q(y + x, q)
        else:
            x = _q(x, q)
            x = self.conv0(x, next(w_iter), fused_modconv=fused_modconv, q16=q, **layer_kwargs)
            x = self.conv1(x, next(w_iter), fused_modconv=fused_modconv, q16=q, **layer_kwargs)
        if img is not None:
            img = upsample2d(img, self.resample_filter)
        if self.is_last or self.architecture == 'skip':
            y = self.torgb(x, next(w_iter), fused_modconv=fused_modconv, q16=q).to(REAL)
            img = img + y if img is not None else y
        return x, img


class SynthesisNetwork(torch.nn.Module):
    """:466-522"""

    def __init__(self, w_dim, img_resolution, img_channels, channel_base=32768, channel_max=512, num_fp16_res=4,
                 **block_kwargs):
        super().__init__()
        self.w_dim, self.img_resolution, self.img_channels = w_dim, img_resolution, img_channels
        log2 = int(np.log2(img_resolution))
        self.block_resolutions = [2 ** i for i in range(2, log2 + 1)]
        ch = {r: min(channel_base // r, channel_max) for r in self.block_resolutions}
        fp16_res = max(2 ** (log2 + 1 - num_fp16_res), 8)
        self.num_ws = 0
        for r in self.block_resolutions:
            block = SynthesisBlock(ch[r // 2] if r > 4 else 0, ch[r], w_dim=w_dim, resolution=r,
                                   img_channels=img_channels, is_last=(r == img_resolution),
                                   use_fp16=(r >= fp16_res), **block_kwargs)
            self.num_ws += block.num_conv
            if r == img_resolution:
                self.num_ws += block.num_torgb
            setattr(self, f'b{r}', block)

    def forward(self, ws, **block_kwargs):
        ws = ws.to(REAL)
        x = img = None
        idx = 0
        for r in self.block_resolutions:
            block = getattr(self, f'b{r}')
            cur = ws.narrow(1, idx, block.num_conv + block.num_torgb)
            idx += block.num_conv
            x, img = block(x, img, cur, **block_kwargs)
        return img


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


class DiscriminatorBlock(torch.nn.Module):
    """:554-639"""

    def __init__(self, in_channels, tmp_channels, out_channels, resolution, img_channels, first_layer_idx,
                 architecture='resnet', activation='lrelu', resample_filter=(1, 3, 3, 1), conv_clamp=None,
                 use_fp16=False, fp16_channels_last=False, freeze_layers=0):
        super().__init__()
        self.in_channels, self.resolution, self.architecture = in_channels, resolution, architecture
        self.use_fp16 = use_fp16
        self.register_buffer('resample_filter', setup_filter(list(resample_filter)))
        self.num_layers = 0

        def trainable():
            t = (first_layer_idx + self.num_layers) >= freeze_layers
            self.num_layers += 1
            return t

        if in_channels == 0 or architecture == 'skip':
            self.fromrgb = Conv2dLayer(img_channels, tmp_channels, kernel_size=1, activation=activation,
                                       trainable=trainable(), conv_clamp=conv_clamp)
        self.conv0 = Conv2dLayer(tmp_channels, tmp_channels, kernel_size=3, activation=activation,
                                 trainable=trainable(), conv_clamp=conv_clamp)
        self.conv1 = Conv2dLayer(tmp_channels, out_channels, kernel_size=3, activation=activation, down=2,
                                 trainable=trainable(), resample_filter=resample_filter, conv_clamp=conv_clamp)
        if architecture == 'resnet':
            self.skip = Conv2dLayer(tmp_channels, out_channels, kernel_size=1, bias=False, down=2,
                                    trainable=trainable(), resample_filter=resample_filter)

    def forward(self, x, img, force_fp32=False):
        q = (self.use_fp16 or EMU16 == torch.float32) and EMU16 is not None and not force_fp32   # :607-608
        x = _q(x, q)
        if self.in_channels == 0 or self.architecture == 'skip':
            y = self.fromrgb(_q(img, q), q16=q)
            x = _q(x + y, q) if x is not None else y
            img = downsample2d(img, self.resample_filter) if self.architecture == 'skip' else None
        if self.architecture == 'resnet':
            y = self.skip(x, gain=np.sqrt(0.5), q16=q)
            x = self.conv0(x, q16=q)
            x = self.conv1(x, gain=np.sqrt(0.5), q16=q)
            x = _q(y + x, q)
        else:
            x = self.conv1(self.conv0(x, q16=q), q16=q)
        return x, img


class MinibatchStdLayer(torch.nn.Module):
    """:643-668"""

    def __init__(self, group_size, num_channels=1):
        super().__init__()
        self.group_size, self.num_channels = group_size, num_channels

    def forward(self, x):
        n, c, h, w = x.shape
        g = min(self.group_size, n) if self.group_size is not None else n
        f = self.num_channels
        y = x.reshape(g, -1, f, c // f, h, w)
        y = y - y.mean(dim=0)
        y = (y.square().mean(dim=0) + 1e-8).sqrt()
        y = y.mean(dim=[2, 3, 4]).reshape(-1, f, 1, 1).repeat(g, 1, h, w)
        return torch.cat([x, y], dim=1)


class DiscriminatorEpilogue(torch.nn.Module):
    """:672-729"""

    def __init__(self, in_channels, cmap_dim, resolution, img_channels, architecture='resnet', mbstd_group_size=4,
                 mbstd_num_channels=1, activation='lrelu', conv_clamp=None):
        super().__init__()
        self.cmap_dim, self.architecture = cmap_dim, architecture
        if architecture == 'skip':
            self.fromrgb = Conv2dLayer(img_channels, in_channels, kernel_size=1, activation=activation)
        self.mbstd = MinibatchStdLayer(mbstd_group_size, mbstd_num_channels) if mbstd_num_channels > 0 else None
        self.conv = Conv2dLayer(in_channels + mbstd_num_channels, in_channels, kernel_size=3, activation=activation,
                                conv_clamp=conv_clamp)
        self.fc = FullyConnectedLayer(in_channels * resolution ** 2, in_channels, activation=activation)
        self.out = FullyConnectedLayer(in_channels, 1 if cmap_dim == 0 else cmap_dim)

    def forward(self, x, img, cmap, force_fp32=False):
        x = x.to(REAL)
        if self.architecture == 'skip':
            x = x + self.fromrgb(img.to(REAL))
        if self.mbstd is not None:
            x = self.mbstd(x)
        x = self.conv(x)
        x = self.out(self.fc(x.flatten(1)))
        if self.cmap_dim > 0:
            x = (x * cmap).sum(dim=1, keepdim=True) * (1 / np.sqrt(self.cmap_dim))
        return x


class Discriminator(torch.nn.Module):
    """:733-792"""

    def __init__(self, c_dim, img_resolution, img_channels, architecture='resnet', channel_base=32768,
                 channel_max=512, num_fp16_res=4, conv_clamp=256, cmap_dim=None, block_kwargs={},
                 mapping_kwargs={}, epilogue_kwargs={}):
        super().__init__()
        self.c_dim, self.img_resolution, self.img_channels = c_dim, img_resolution, img_channels
        log2 = int(np.log2(img_resolution))
        self.block_resolutions = [2 ** i for i in range(log2, 2, -1)]
        ch = {r: min(channel_base // r, channel_max) for r in self.block_resolutions + [4]}
        fp16_res = max(2 ** (log2 + 1 - num_fp16_res), 8)
        if cmap_dim is None:
            cmap_dim = ch[4]
        if c_dim == 0:
            cmap_dim = 0
        common = dict(img_channels=img_channels, architecture=architecture, conv_clamp=conv_clamp)
        idx = 0
        for r in self.block_resolutions:
            block = DiscriminatorBlock(ch[r] if r < img_resolution else 0, ch[r], ch[r // 2], resolution=r,
                                       first_layer_idx=idx, use_fp16=(r >= fp16_res), **block_kwargs, **common)
            setattr(self, f'b{r}', block)
            idx += block.num_layers
        if c_dim > 0:
            self.mapping = MappingNetwork(z_dim=0, c_dim=c_dim, w_dim=cmap_dim, num_ws=None, w_avg_beta=None,
                                          **mapping_kwargs)
        self.b4 = DiscriminatorEpilogue(ch[4], cmap_dim=cmap_dim, resolution=4, **epilogue_kwargs, **common)

    def forward(self, img, c, update_emas=False, **block_kwargs):
        x = None
        for r in self.block_resolutions:
            x, img = getattr(self, f'b{r}')(x, img, **block_kwargs)
        cmap = self.mapping(None, c) if self.c_dim > 0 else None
        return self.b4(x, img, cmap)


# =============================================================================================
# ADA augmentation pipe  (SG3/training/augment_mi.py:30-453)
# =============================================================================================

WAVELETS = {
    'sym2': [-0.12940952255092145, 0.22414386804185735, 0.836516303737469, 0.48296291314469025],
    'sym6': [0.015404109327027373, 0.0034907120842174702, -0.11799011114819057, -0.048311742585633,
             0.4910559419267466, 0.787641141030194, 0.3379294217276218, -0.07263752278646252,
             -0.021060292512300564, 0.04472490177066578, 0.0017677118642428036, -0.007800708325034148],
}


def _mat(*rows):
    """Batched homogeneous matrix from rows of tensors/scalars (augment_mi.py:52-60)."""
    ref = [v for r in rows for v in r if isinstance(v, torch.Tensor)]
    if not ref:
        return torch.tensor(np.asarray(rows), dtype=REAL)
    shape = ref[0].shape
    elems = [v if isinstance(v, torch.Tensor) else torch.full(shape, float(v)) for r in rows for v in r]
    return torch.stack(elems, dim=-1).reshape(*shape, len(rows), -1)


def translate2d(tx, ty):
    return _mat([1, 0, tx], [0, 1, ty], [0, 0, 1])


def scale2d(sx, sy):
    return _mat([sx, 0, 0], [0, sy, 0], [0, 0, 1])


def rotate2d(t):
    return _mat([torch.cos(t), torch.sin(-t), 0], [torch.sin(t), torch.cos(t), 0], [0, 0, 1])


def translate3d(tx, ty, tz):
    return _mat([1, 0, 0, tx], [0, 1, 0, ty], [0, 0, 1, tz], [0, 0, 0, 1])


def scale3d(sx, sy, sz):
    return _mat([sx, 0, 0, 0], [0, sy, 0, 0], [0, 0, sz, 0], [0, 0, 0, 1])


def rotate3d(v, t):
    vx, vy, vz = v[..., 0], v[..., 1], v[..., 2]
    s, c = torch.sin(t), torch.cos(t)
    cc = 1 - c
    return _mat([vx * vx * cc + c, vx * vy * cc - vz * s, vx * vz * cc + vy * s, 0],
                [vy * vx * cc + vz * s, vy * vy * cc + c, vy * vz * cc - vx * s, 0],
                [vz * vx * cc - vy * s, vz * vy * cc + vx * s, vz * vz * cc + c, 0],
                [0, 0, 0, 1])


def _filter_bank():
    """augment_mi.py:186-195 (no scipy: full 1-D convolution by numpy)."""
    lo = np.asarray(WAVELETS['sym2'])
    hi = lo * ((-1) ** np.arange(lo.size))
    lo2 = np.convolve(lo, lo[::-1]) / 2
    hi2 = np.convolve(hi, hi[::-1]) / 2
    fb = np.eye(4, 1)
    for i in range(1, fb.shape[0]):
        fb = np.dstack([fb, np.zeros_like(fb)]).reshape(fb.shape[0], -1)[:, :-1]
        fb = np.stack([np.convolve(row, lo2) for row in fb])
        a = (fb.shape[1] - hi2.size) // 2
        fb[i, a: a + hi2.size] += hi2
    return fb


class AugmentPipe(torch.nn.Module):
    def __init__(self, run_dir=None, batch_size=None, xflip=0, rotate90=0, xint=0, xint_max=0.125,
                 scale=0, rotate=0, aniso=0, xfrac=0, scale_std=0.2, rotate_max=1, aniso_std=0.2, xfrac_std=0.125,
                 brightness=0, contrast=0, lumaflip=0, hue=0, saturation=0, brightness_std=0.2, contrast_std=0.5,
                 hue_max=1, saturation_std=1, imgfilter=0, imgfilter_bands=(1, 1, 1, 1), imgfilter_std=1,
                 noise=0, cutout=0, noise_std=0.1, cutout_size=0.5):
        super().__init__()
        self.register_buffer('p', torch.ones([]))
        for k, v in dict(xflip=xflip, rotate90=rotate90, xint=xint, xint_max=xint_max, scale=scale, rotate=rotate,
                         aniso=aniso, xfrac=xfrac, scale_std=scale_std, rotate_max=rotate_max, aniso_std=aniso_std,
                         xfrac_std=xfrac_std, brightness=brightness, contrast=contrast, lumaflip=lumaflip, hue=hue,
                         saturation=saturation, brightness_std=brightness_std, contrast_std=contrast_std,
                         hue_max=hue_max, saturation_std=saturation_std, imgfilter=imgfilter,
                         imgfilter_std=imgfilter_std, noise=noise, cutout=cutout, noise_std=noise_std,
                         cutout_size=cutout_size).items():
            setattr(self, k, float(v))
        self.imgfilter_bands = list(imgfilter_bands)
        self.register_buffer('Hz_geom', setup_filter(WAVELETS['sym6']))
        self.register_buffer('Hz_fbank', torch.as_tensor(_filter_bank(), dtype=REAL))

    def forward(self, images, allow_aug_debug_print=False, debug_percentile=None):
        n, c, h, w = images.shape
        dp = None if debug_percentile is None else torch.as_tensor(debug_percentile, dtype=REAL)
        I3 = torch.eye(3)
        G = I3
        if self.xflip > 0:                                                       # :213-218
            i = torch.floor(torch.rand([n]) * 2)
            i = torch.where(torch.rand([n]) < self.xflip * self.p, i, torch.zeros_like(i))
            if dp is not None:
                i = torch.full_like(i, torch.floor(dp * 2))
            G = G @ scale2d(1 / (1 - 2 * i), 1)
        if self.rotate90 > 0:                                                    # :221-226
            i = torch.floor(torch.rand([n]) * 4)
            i = torch.where(torch.rand([n]) < self.rotate90 * self.p, i, torch.zeros_like(i))
            if dp is not None:
                i = torch.full_like(i, torch.floor(dp * 4))
            G = G @ rotate2d(np.pi / 2 * i)
        if self.xint > 0:                                                        # :229-234
            t = (torch.rand([n, 2]) * 2 - 1) * self.xint_max
            t = torch.where(torch.rand([n, 1]) < self.xint * self.p, t, torch.zeros_like(t))
            if dp is not None:
                t = torch.full_like(t, (dp * 2 - 1) * self.xint_max)
            G = G @ translate2d(-torch.round(t[:, 0] * w), -torch.round(t[:, 1] * h))
        if self.scale > 0:                                                       # :241-246
            s = torch.exp2(torch.randn([n]) * self.scale_std)
            s = torch.where(torch.rand([n]) < self.scale * self.p, s, torch.ones_like(s))
            if dp is not None:
                s = torch.full_like(s, torch.exp2(torch.erfinv(dp * 2 - 1) * self.scale_std))
            G = G @ scale2d(1 / s, 1 / s)
        p_rot = 1 - torch.sqrt((1 - self.rotate * self.p).clamp(0, 1))           # :249
        if self.rotate > 0:                                                      # :250-255
            th = (torch.rand([n]) * 2 - 1) * np.pi * self.rotate_max
            th = torch.where(torch.rand([n]) < p_rot, th, torch.zeros_like(th))
            if dp is not None:
                th = torch.full_like(th, (dp * 2 - 1) * np.pi * self.rotate_max)
            G = G @ rotate2d(th)
        if self.aniso > 0:                                                       # :258-263
            s = torch.exp2(torch.randn([n]) * self.aniso_std)
            s = torch.where(torch.rand([n]) < self.aniso * self.p, s, torch.ones_like(s))
            if dp is not None:
                s = torch.full_like(s, torch.exp2(torch.erfinv(dp * 2 - 1) * self.aniso_std))
            G = G @ scale2d(1 / s, s)
        if self.rotate > 0:                                                      # :266-271
            th = (torch.rand([n]) * 2 - 1) * np.pi * self.rotate_max
            th = torch.where(torch.rand([n]) < p_rot, th, torch.zeros_like(th))
            if dp is not None:
                th = torch.zeros_like(th)
            G = G @ rotate2d(th)
        if self.xfrac > 0:                                                       # :274-279
            t = torch.randn([n, 2]) * self.xfrac_std
            t = torch.where(torch.rand([n, 1]) < self.xfrac * self.p, t, torch.zeros_like(t))
            if dp is not None:
                t = torch.full_like(t, torch.erfinv(dp * 2 - 1) * self.xfrac_std)
            G = G @ translate2d(-t[:, 0] * w, -t[:, 1] * h)

        if G is not I3:                                                          # :286-321
            cx, cy = (w - 1) / 2, (h - 1) / 2
            cp = _mat([-cx, -cy, 1], [cx, -cy, 1], [cx, cy, 1], [-cx, cy, 1])
            cp = G @ cp.t()
            hz_pad = self.Hz_geom.shape[0] // 4
            margin = cp[:, :2, :].permute(1, 0, 2).flatten(1)
            margin = torch.cat([-margin, margin]).max(dim=1).values
            margin = margin + torch.tensor([hz_pad * 2 - cx, hz_pad * 2 - cy] * 2, dtype=REAL)
            margin = margin.max(torch.tensor([0, 0] * 2, dtype=REAL))
            margin = margin.min(torch.tensor([w - 1, h - 1] * 2, dtype=REAL))
            mx0, my0, mx1, my1 = [int(v) for v in margin.ceil().to(torch.int32)]
            images = F.pad(images, [mx0, mx1, my0, my1], mode='reflect')
            G = translate2d((mx0 - mx1) / 2, (my0 - my1) / 2) @ G
            images = upsample2d(images, self.Hz_geom, up=2)
            G = scale2d(2, 2) @ G @ scale2d(1 / 2, 1 / 2)
            G = translate2d(-0.5, -0.5) @ G @ translate2d(0.5, 0.5)
            shape = [n, c, (h + hz_pad * 2) * 2, (w + hz_pad * 2) * 2]
            G = scale2d(2 / images.shape[3], 2 / images.shape[2]) @ G @ scale2d(1 / (2 / shape[3]), 1 / (2 / shape[2]))
            grid = F.affine_grid(G[:, :2, :], shape, align_corners=False)
            images = grid_sample(images, grid)
            images = downsample2d(images, self.Hz_geom, down=2, padding=-hz_pad * 2, flip_filter=True)

        I4 = torch.eye(4)
        C = I4
        if self.brightness > 0:                                                  # :332-337
            b = torch.randn([n]) * self.brightness_std
            b = torch.where(torch.rand([n]) < self.brightness * self.p, b, torch.zeros_like(b))
            if dp is not None:
                b = torch.full_like(b, torch.erfinv(dp * 2 - 1) * self.brightness_std)
            C = translate3d(b, b, b) @ C
        if self.contrast > 0:                                                    # :340-345
            k = torch.exp2(torch.randn([n]) * self.contrast_std)
            k = torch.where(torch.rand([n]) < self.contrast * self.p, k, torch.ones_like(k))
            if dp is not None:
                k = torch.full_like(k, torch.exp2(torch.erfinv(dp * 2 - 1) * self.contrast_std))
            C = scale3d(k, k, k) @ C
        v = torch.tensor(np.asarray([1, 1, 1, 0]) / np.sqrt(3), dtype=REAL)
        if self.lumaflip > 0:                                                    # :349-354
            i = torch.floor(torch.rand([n, 1, 1]) * 2)
            i = torch.where(torch.rand([n, 1, 1]) < self.lumaflip * self.p, i, torch.zeros_like(i))
            if dp is not None:
                i = torch.full_like(i, torch.floor(dp * 2))
            C = (I4 - 2 * torch.outer(v, v) * i) @ C
        if self.hue > 0 and c > 1:                                               # :357-362
            th = (torch.rand([n]) * 2 - 1) * np.pi * self.hue_max
            th = torch.where(torch.rand([n]) < self.hue * self.p, th, torch.zeros_like(th))
            if dp is not None:
                th = torch.full_like(th, (dp * 2 - 1) * np.pi * self.hue_max)
            C = rotate3d(v, th) @ C
        if self.saturation > 0 and c > 1:                                        # :365-370
            s = torch.exp2(torch.randn([n, 1, 1]) * self.saturation_std)
            s = torch.where(torch.rand([n, 1, 1]) < self.saturation * self.p, s, torch.ones_like(s))
            if dp is not None:
                s = torch.full_like(s, torch.exp2(torch.erfinv(dp * 2 - 1) * self.saturation_std))
            C = (torch.outer(v, v) + (I4 - torch.outer(v, v)) * s) @ C
        if C is not I4:                                                          # :377-386
            images = images.reshape(n, c, h * w)
            if c == 3:
                images = C[:, :3, :3] @ images + C[:, :3, 3:]
            elif c == 1:
                Cm = C[:, :3, :].mean(dim=1, keepdim=True)
                images = images * Cm[:, :, :3].sum(dim=2, keepdim=True) + Cm[:, :, 3:]
            else:
                raise ValueError('Image must be RGB (3 channels) or L (1 channel)')
            images = images.reshape(n, c, h, w)

        if self.imgfilter > 0:                                                   # :392-420
            nb = self.Hz_fbank.shape[0]
            power = torch.tensor(np.array([10, 1, 1, 1]) / 13, dtype=REAL)
            g = torch.ones([n, nb])
            for i, bs in enumerate(self.imgfilter_bands):
                ti = torch.exp2(torch.randn([n]) * self.imgfilter_std)
                ti = torch.where(torch.rand([n]) < self.imgfilter * self.p * bs, ti, torch.ones_like(ti))
                if dp is not None:
                    ti = torch.full_like(ti, torch.exp2(torch.erfinv(dp * 2 - 1) * self.imgfilter_std)) \
                        if bs > 0 else torch.ones_like(ti)
                t = torch.ones([n, nb])
                t[:, i] = ti
                t = t / (power * t.square()).sum(dim=-1, keepdim=True).sqrt()
                g = g * t
            hz = (g @ self.Hz_fbank).unsqueeze(1).repeat([1, c, 1]).reshape(n * c, 1, -1)
            p = self.Hz_fbank.shape[1] // 2
            images = F.pad(images.reshape(1, n * c, h, w), [p, p, p, p], mode='reflect')
            images = F.conv2d(images, hz.unsqueeze(2), groups=n * c)
            images = F.conv2d(images, hz.unsqueeze(3), groups=n * c)
            images = images.reshape(n, c, h, w)

        if self.noise > 0:                                                       # :427-432
            sigma = torch.randn([n, 1, 1, 1]).abs() * self.noise_std
            sigma = torch.where(torch.rand([n, 1, 1, 1]) < self.noise * self.p, sigma, torch.zeros_like(sigma))
            if dp is not None:
                sigma = torch.full_like(sigma, torch.erfinv(dp) * self.noise_std)
            images = images + torch.randn([n, c, h, w]) * sigma
        if self.cutout > 0:                                                      # :435-447
            size = torch.full([n, 2, 1, 1, 1], self.cutout_size)
            size = torch.where(torch.rand([n, 1, 1, 1, 1]) < self.cutout * self.p, size, torch.zeros_like(size))
            center = torch.rand([n, 2, 1, 1, 1])
            if dp is not None:
                size = torch.full_like(size, self.cutout_size)
                center = torch.full_like(center, dp)
            cx_ = torch.arange(w).reshape(1, 1, 1, -1)
            cy_ = torch.arange(h).reshape(1, 1, -1, 1)
            mx = ((cx_ + 0.5) / w - center[:, 0]).abs() >= size[:, 0] / 2
            my = ((cy_ + 0.5) / h - center[:, 1]).abs() >= size[:, 1] / 2
            images = images * torch.logical_or(mx, my).to(REAL)
        return images


# =============================================================================================
# loss  (SG3/training/loss.py:23-139)
# =============================================================================================


class StyleGAN2Loss:
    def __init__(self, device, G, D, augment_pipe=None, r1_gamma=10, style_mixing_prob=0, pl_weight=0,
                 pl_batch_shrink=2, pl_decay=0.01, pl_no_weight_grad=False, blur_init_sigma=0, blur_fade_kimg=0,
                 allow_aug_debug_print=False, report=None):
        self.G, self.D, self.augment_pipe = G, D, augment_pipe
        self.r1_gamma, self.style_mixing_prob = r1_gamma, style_mixing_prob
        self.pl_weight, self.pl_batch_shrink, self.pl_decay = pl_weight, pl_batch_shrink, pl_decay
        self.pl_mean = torch.zeros([])
        self.blur_init_sigma, self.blur_fade_kimg = blur_init_sigma, blur_fade_kimg
        self.report = report if report is not None else (lambda name, value: value)

    def run_G(self, z, c, update_emas=False):
        ws = self.G.mapping(z, c, update_emas=update_emas)
        if self.style_mixing_prob > 0:
            cutoff = torch.empty([], dtype=torch.int64).random_(1, ws.shape[1])
            cutoff = torch.where(torch.rand([]) < self.style_mixing_prob, cutoff, torch.full_like(cutoff, ws.shape[1]))
            ws[:, cutoff:] = self.G.mapping(torch.randn_like(z), c, update_emas=False)[:, cutoff:]
        return self.G.synthesis(ws, update_emas=update_emas), ws

    def run_D(self, img, c, blur_sigma=0, update_emas=False):
        size = np.floor(blur_sigma * 3)
        if size > 0:
            f = torch.arange(-size, size + 1).div(blur_sigma).square().neg().exp2()
            img = filter2d(img, f / f.sum())
        if self.augment_pipe is not None:
            img = self.augment_pipe(img, False)
        return self.D(img, c, update_emas=update_emas)

    def accumulate_gradients(self, phase, real_img, real_c, gen_z, gen_c, gain, cur_nimg):
        if self.pl_weight == 0:
            phase = {'Greg': 'none', 'Gboth': 'Gmain'}.get(phase, phase)
        if self.r1_gamma == 0:
            phase = {'Dreg': 'none', 'Dboth': 'Dmain'}.get(phase, phase)
        blur = max(1 - cur_nimg / (self.blur_fade_kimg * 1e3), 0) * self.blur_init_sigma if self.blur_fade_kimg > 0 else 0
        rep = self.report
        if phase in ['Gmain', 'Gboth']:
            img, _ = self.run_G(gen_z, gen_c)
            logits = self.run_D(img, gen_c, blur_sigma=blur)
            rep('Loss/scores/fake', logits)
            rep('Loss/signs/fake', logits.sign())
            loss = F.softplus(-logits)
            rep('Loss/G/loss', loss)
            loss.mean().mul(gain).backward()
        if phase in ['Greg', 'Gboth']:
            bs = gen_z.shape[0] // self.pl_batch_shrink
            img, ws = self.run_G(gen_z[:bs], gen_c[:bs])
            pl_noise = torch.randn_like(img) / np.sqrt(img.shape[2] * img.shape[3])
            pl_grads = torch.autograd.grad([(img * pl_noise).sum()], [ws], create_graph=True, only_inputs=True)[0]
            pl_len = pl_grads.square().sum(2).mean(1).sqrt()
            pl_mean = self.pl_mean.lerp(pl_len.mean(), self.pl_decay)
            self.pl_mean.copy_(pl_mean.detach())
            pen = (pl_len - pl_mean).square()
            rep('Loss/pl_penalty', pen)
            loss = pen * self.pl_weight
            rep('Loss/G/reg', loss)
            loss.mean().mul(gain).backward()
        loss_gen = 0
        if phase in ['Dmain', 'Dboth']:
            img, _ = self.run_G(gen_z, gen_c, update_emas=True)
            logits = self.run_D(img, gen_c, blur_sigma=blur, update_emas=True)
            rep('Loss/scores/fake', logits)
            rep('Loss/signs/fake', logits.sign())
            loss_gen = F.softplus(logits)
            loss_gen.mean().mul(gain).backward()
        if phase in ['Dmain', 'Dreg', 'Dboth']:
            real = real_img.detach().requires_grad_(phase in ['Dreg', 'Dboth'])
            logits = self.run_D(real, real_c, blur_sigma=blur)
            rep('Loss/scores/real', logits)
            rep('Loss/signs/real', logits.sign())
            loss_real = 0
            if phase in ['Dmain', 'Dboth']:
                loss_real = F.softplus(-logits)
                rep('Loss/D/loss', loss_gen + loss_real)
            loss_r1 = 0
            if phase in ['Dreg', 'Dboth']:
                g = torch.autograd.grad([logits.sum()], [real], create_graph=True, only_inputs=True)[0]
                pen = g.square().sum([1, 2, 3])
                loss_r1 = pen * (self.r1_gamma / 2)
                rep('Loss/r1_penalty', pen)
                rep('Loss/D/reg', loss_r1)
            (loss_real + loss_r1).mean().mul(gain).backward()


# =============================================================================================
# one training iteration  (SG3/training/training_loop_mi_multimodal.py:243-366, single process)
# =============================================================================================


def make_phases(G, D, G_reg_interval=4, D_reg_interval=16, glr=0.0025, dlr=0.0025, betas=(0, 0.99), eps=1e-8):
    phases = []
    for name, module, reg, lr in [('G', G, G_reg_interval, glr), ('D', D, D_reg_interval, dlr)]:
        r = reg / (reg + 1)
        opt = torch.optim.Adam(module.parameters(), lr=lr * r, betas=[b ** r for b in betas], eps=eps)
        phases += [dict(name=name + 'main', module=module, opt=opt, interval=1),
                   dict(name=name + 'reg', module=module, opt=opt, interval=reg)]
    return phases


def D_of(phases):
    return next(ph['module'] for ph in phases if ph['name'].startswith('D'))


def train_iteration(loss, phases, G, G_ema, real_img, real_c, all_gen_z, all_gen_c, batch_idx, cur_nimg,
                    batch_size, ema_kimg=10, ema_rampup=0.05, on_grads=None, isolated=False):
    """isolated: every phase starts from the state the iteration started from (parameters and buffers restored,
    no optimiser step, no EMA) -- the phase-isolated form of the parity fixtures (tests/golden/make_golden.py
    gen_config_isolated): each phase's gradients are then a function of one fixed state, not of the earlier
    phases' Adam steps (whose first step, beta1 = 0, is ~lr * sign(g) for every gradient entry)."""
    start = None
    if isolated:
        start = [{k: v.detach().clone() for k, v in m.state_dict().items()} for m in (G, D_of(phases))]
    for pi, ph in enumerate(phases):
        if batch_idx % ph['interval'] != 0:
            continue
        if isolated:
            with torch.no_grad():
                for m, sd in zip((G, D_of(phases)), start):
                    for k, v in m.state_dict().items():
                        v.copy_(sd[k])
        ph['opt'].zero_grad(set_to_none=True)
        ph['module'].requires_grad_(True)
        loss.accumulate_gradients(ph['name'], real_img, real_c, all_gen_z[pi], all_gen_c[pi], ph['interval'], cur_nimg)
        ph['module'].requires_grad_(False)
        params = [p for p in ph['module'].parameters() if p.grad is not None]
        if params:
            flat = torch.cat([p.grad.flatten() for p in params])
            torch.nan_to_num(flat, nan=0, posinf=1e5, neginf=-1e5, out=flat)
            for p, g in zip(params, flat.split([p.numel() for p in params])):
                p.grad = g.reshape(p.shape)
            if on_grads is not None:
                on_grads(ph['name'], ph['module'])
        if not isolated:
            ph['opt'].step()
    if isolated:
        return None
    ema_nimg = ema_kimg * 1000
    if ema_rampup is not None:
        ema_nimg = min(ema_nimg, cur_nimg * ema_rampup)
    beta = 0.5 ** (batch_size / max(ema_nimg, 1e-8))
    with torch.no_grad():
        for pe, p in zip(G_ema.parameters(), G.parameters()):
            pe.copy_(p.lerp(pe, beta))
        for be, b in zip(G_ema.buffers(), G.buffers()):
            be.copy_(b)
    return beta


def clone_module(m):
    return copy.deepcopy(m)
