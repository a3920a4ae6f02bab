"""Differentiable ADA augmentation pipe on the MI355X kernels.

Drop-in for SG3/training/augment_mi.py:125-453 (`AugmentPipe(run_dir, batch_size, **probs)`,
`forward(images, allow_aug_debug_print, debug_percentile=None)`, `p` buffer).  The geometric
stage -- reflect pad, 2x upsample with the 12-tap sym6 filter, bilinear warp, 2x downsample --
runs on sg2_upfirdn2d (separable, taps in LDS) and sg2_grid_sample (fwd + input gradient, whose
backward is again the forward, so R1's double backward stays on the kernels).  Per-sample 3x3 / 4x4
transform matrices are tiny and built with torch ops on the device, drawing random numbers in the
reference's order (so an RNG tape reproduces the reference exactly).

Deviation: `allow_aug_debug_print` (matplotlib PNG dump, :449-491) is accepted and ignored.
"""
import ctypes

import numpy as np
import torch

import sg2hip as _hip
from torch_utils import misc
from torch_utils import persistence
from torch_utils.ops import conv2d_gradfix
from torch_utils.ops import grid_sample_gradfix
from torch_utils.ops import reflect_pad
from torch_utils.ops import upfirdn2d

# the transform algebra of the geometric stage in one launch (sg2_aug_geom); False: the per-op torch algebra
# (debug-percentile mode always takes it)
fused_geometric = True

wavelets = {
    'haar': [0.7071067811865476, 0.7071067811865476],
    'db1': [0.7071067811865476, 0.7071067811865476],
    'sym2': [-0.12940952255092145, 0.22414386804185735, 0.836516303737469, 0.48296291314469025],
    'sym6': [0.015404109327027373, 0.0034907120842174702, -0.11799011114819057, -0.048311742585633,
             0.4910559419267466, 0.787641141030194, 0.3379294217276218, -0.07263752278646252,
             -0.021060292512300564, 0.04472490177066578, 0.0017677118642428036, -0.007800708325034148],
}


def matrix(*rows, device=None):
    """Stack scalar / per-sample entries into [..., R, C] matrices (reference :52-60)."""
    assert all(len(r) == len(rows[0]) for r in rows)
    elems = [v for r in rows for v in r]
    ref = [v for v in elems if isinstance(v, torch.Tensor)]
    if not ref:
        return misc.constant(np.asarray(rows), device=device)
    shape, dev = ref[0].shape, ref[0].device
    elems = [v if isinstance(v, torch.Tensor) else misc.constant(v, shape=shape, device=dev) for v in elems]
    return torch.stack(elems, dim=-1).reshape(shape + (len(rows), -1))


def translate2d(tx, ty, **kw):
    return matrix([1, 0, tx], [0, 1, ty], [0, 0, 1], **kw)


def translate3d(tx, ty, tz, **kw):
    return matrix([1, 0, 0, tx], [0, 1, 0, ty], [0, 0, 1, tz], [0, 0, 0, 1], **kw)


def scale2d(sx, sy, **kw):
    return matrix([sx, 0, 0], [0, sy, 0], [0, 0, 1], **kw)


def scale3d(sx, sy, sz, **kw):
    return matrix([sx, 0, 0, 0], [0, sy, 0, 0], [0, 0, sz, 0], [0, 0, 0, 1], **kw)


def rotate2d(theta, **kw):
    return matrix([torch.cos(theta), torch.sin(-theta), 0], [torch.sin(theta), torch.cos(theta), 0], [0, 0, 1], **kw)


def rotate3d(v, theta, **kw):
    vx, vy, vz = v[..., 0], v[..., 1], v[..., 2]
    s, c = torch.sin(theta), torch.cos(theta)
    cc = 1 - c
    return matrix([vx * vx * cc + c, vx * vy * cc - vz * s, vx * vz * cc + vy * s, 0],
                  [vy * vx * cc + vz * s, vy * vy * cc + c, vy * vz * cc - vx * s, 0],
                  [vz * vx * cc - vy * s, vz * vy * cc + vx * s, vz * vz * cc + c, 0],
                  [0, 0, 0, 1], **kw)


def translate2d_inv(tx, ty, **kw):
    return translate2d(-tx, -ty, **kw)


def scale2d_inv(sx, sy, **kw):
    return scale2d(1 / sx, 1 / sy, **kw)


def rotate2d_inv(theta, **kw):
    return rotate2d(-theta, **kw)


def _filter_bank():
    """Image-space filter bank of the reference (:186-195) built with numpy only."""
    lo = np.asarray(wavelets['sym2'])
    hi = lo * ((-1) ** np.arange(lo.size))
    lo2 = np.convolve(lo, lo[::-1]) / 2
    hi2 = np.convolve(hi, hi[::-1]) / 2
    fb = np.eye(4, 1)
    for i in range(1, fb.shape[0]):
        fb = np.dstack([fb, np.zeros_like(fb)]).reshape(fb.shape[0], -1)[:, :-1]
        fb = np.stack([np.convolve(row, lo2) for row in fb])
        start = (fb.shape[1] - hi2.size) // 2
        fb[i, start:start + hi2.size] += hi2
    return fb


@persistence.persistent_class
class AugmentPipe(torch.nn.Module):
    def __init__(self, run_dir=None, batch_size=None,
                 xflip=0, rotate90=0, xint=0, xint_max=0.125,
                 scale=0, rotate=0, aniso=0, xfrac=0, scale_std=0.2, rotate_max=1, aniso_std=0.2, xfrac_std=0.125,
                 brightness=0, contrast=0, lumaflip=0, hue=0, saturation=0, brightness_std=0.2, contrast_std=0.5,
                 hue_max=1, saturation_std=1,
                 imgfilter=0, imgfilter_bands=[1, 1, 1, 1], imgfilter_std=1,
                 noise=0, cutout=0, noise_std=0.1, cutout_size=0.5):
        super().__init__()
        self.register_buffer('p', torch.ones([]))
        self.xflip, self.rotate90, self.xint, self.xint_max = float(xflip), float(rotate90), float(xint), float(xint_max)
        self.scale, self.rotate, self.aniso, self.xfrac = float(scale), float(rotate), float(aniso), float(xfrac)
        self.scale_std, self.rotate_max = float(scale_std), float(rotate_max)
        self.aniso_std, self.xfrac_std = float(aniso_std), float(xfrac_std)
        self.brightness, self.contrast, self.lumaflip = float(brightness), float(contrast), float(lumaflip)
        self.hue, self.saturation = float(hue), float(saturation)
        self.brightness_std, self.contrast_std = float(brightness_std), float(contrast_std)
        self.hue_max, self.saturation_std = float(hue_max), float(saturation_std)
        self.imgfilter, self.imgfilter_bands, self.imgfilter_std = float(imgfilter), list(imgfilter_bands), float(imgfilter_std)
        self.noise, self.cutout, self.noise_std, self.cutout_size = float(noise), float(cutout), float(noise_std), float(cutout_size)
        self.run_dir, self.batch_size = run_dir, batch_size
        self.register_buffer('Hz_geom', upfirdn2d.setup_filter(wavelets['sym6']))
        self.register_buffer('Hz_fbank', torch.as_tensor(_filter_bank(), dtype=torch.float32))

    # ------------------------------------------------------------------ geometric
    def _geometric_enabled(self):
        return any(v > 0 for v in (self.xflip, self.rotate90, self.xint, self.scale, self.rotate, self.aniso,
                                   self.xfrac))

    def _geometric_fused(self, images):
        """The geometric stage with the transform algebra in one launch (sg2_aug_geom): the same draws, in the
        same order, as _geometric below; the kernel composes each sample's matrix, the batch margins and the
        pad / up-sampling conjugations (reference :214-318) that _geometric builds with ~100 small torch ops."""
        n, c, h, w = images.shape
        dev = images.device
        rand = lambda *s: torch.rand(list(s), device=dev)    # noqa: E731
        randn = lambda *s: torch.randn(list(s), device=dev)  # noqa: E731
        draws = [None] * 16
        if self.xflip > 0:
            draws[0], draws[1] = rand(n), rand(n)
        if self.rotate90 > 0:
            draws[2], draws[3] = rand(n), rand(n)
        if self.xint > 0:
            draws[4], draws[5] = rand(n, 2), rand(n, 1)
        if self.scale > 0:
            draws[6], draws[7] = randn(n), rand(n)
        if self.rotate > 0:
            draws[8], draws[9] = rand(n), rand(n)
        if self.aniso > 0:
            draws[10], draws[11] = randn(n), rand(n)
        if self.rotate > 0:
            draws[12], draws[13] = rand(n), rand(n)
        if self.xfrac > 0:
            draws[14], draws[15] = randn(n, 2), rand(n, 1)
        hz_pad = self.Hz_geom.shape[0] // 4
        hup, wup = (h + hz_pad * 2) * 2, (w + hz_pad * 2) * 2
        theta = torch.empty([n, 2, 3], dtype=torch.float32, device=dev)
        ints = torch.empty([14], dtype=torch.int32, device=dev)          # margins [4], lims [8], dyn_hw [2]
        mi, lims, dyn_hw = ints[:4], ints[4:12], ints[12:]
        a = _hip.AugGeomArgs()
        for k, t in enumerate(draws):
            a.draw[k] = _hip.ptr(t)
        a.p = _hip.ptr(self.p)
        for k in ('xflip', 'rotate90', 'xint', 'xint_max', 'scale', 'rotate', 'aniso', 'xfrac', 'scale_std',
                  'rotate_max', 'aniso_std', 'xfrac_std'):
            setattr(a, k, getattr(self, k))
        a.pad_x, a.pad_y = hz_pad * 2 - (w - 1) / 2, hz_pad * 2 - (h - 1) / 2
        a.inv_sx, a.inv_sy = 1 / (2 / wup), 1 / (2 / hup)
        a.n, a.h, a.w = n, h, w
        _hip.check(_hip.lib().sg2_aug_geom(_hip.ptr(theta), _hip.ptr(mi), _hip.ptr(lims), _hip.ptr(dyn_hw),
                                           ctypes.byref(a), _hip.stream_ptr(dev)), 'sg2_aug_geom')
        images = reflect_pad.reflect_pad_dyn(images, mi)
        images = upfirdn2d.upsample2d_limited(images, self.Hz_geom, lims.view(4, 2).unbind(0), up=2)
        images = grid_sample_gradfix.affine_grid_sample(images, theta, [n, c, hup, wup], dyn_hw=dyn_hw)
        return upfirdn2d.downsample2d(x=images, f=self.Hz_geom, down=2, padding=-hz_pad * 2, flip_filter=True)

    def _geometric(self, images, dp):
        n, c, h, w = images.shape
        dev = images.device
        if dp is None and images.is_cuda and fused_geometric and self._geometric_enabled():
            return self._geometric_fused(images)
        I_3 = torch.eye(3, device=dev)
        G = I_3

        def choose(prob, val, alt, shape):
            return torch.where(torch.rand(shape, device=dev) < prob, val, alt)

        if self.xflip > 0:
            i = torch.floor(torch.rand([n], device=dev) * 2)
            i = choose(self.xflip * self.p, i, torch.zeros_like(i), [n])
            if dp is not None:
                i = torch.full_like(i, torch.floor(dp * 2))
            G = G @ scale2d_inv(1 - 2 * i, 1)
        if self.rotate90 > 0:
            i = torch.floor(torch.rand([n], device=dev) * 4)
            i = choose(self.rotate90 * self.p, i, torch.zeros_like(i), [n])
            if dp is not None:
                i = torch.full_like(i, torch.floor(dp * 4))
            G = G @ rotate2d_inv(-np.pi / 2 * i)
        if self.xint > 0:
            t = (torch.rand([n, 2], device=dev) * 2 - 1) * self.xint_max
            t = choose(self.xint * self.p, t, torch.zeros_like(t), [n, 1])
            if dp is not None:
                t = torch.full_like(t, (dp * 2 - 1) * self.xint_max)
            G = G @ translate2d_inv(torch.round(t[:, 0] * w), torch.round(t[:, 1] * h))
        if self.scale > 0:
            s = torch.exp2(torch.randn([n], device=dev) * self.scale_std)
            s = choose(self.scale * self.p, s, torch.ones_like(s), [n])
            if dp is not None:
                s = torch.full_like(s, torch.exp2(torch.erfinv(dp * 2 - 1) * self.scale_std))
            G = G @ scale2d_inv(s, s)
        p_rot = 1 - torch.sqrt((1 - self.rotate * self.p).clamp(0, 1))
        if self.rotate > 0:
            th = (torch.rand([n], device=dev) * 2 - 1) * np.pi * self.rotate_max
            th = choose(p_rot, th, torch.zeros_like(th), [n])
            if dp is not None:
                th = torch.full_like(th, (dp * 2 - 1) * np.pi * self.rotate_max)
            G = G @ rotate2d_inv(-th)
        if self.aniso > 0:
            s = torch.exp2(torch.randn([n], device=dev) * self.aniso_std)
            s = choose(self.aniso * self.p, s, torch.ones_like(s), [n])
            if dp is not None:
                s = torch.full_like(s, torch.exp2(torch.erfinv(dp * 2 - 1) * self.aniso_std))
            G = G @ scale2d_inv(s, 1 / s)
        if self.rotate > 0:
            th = (torch.rand([n], device=dev) * 2 - 1) * np.pi * self.rotate_max
            th = choose(p_rot, th, torch.zeros_like(th), [n])
            if dp is not None:
                th = torch.zeros_like(th)
            G = G @ rotate2d_inv(-th)
        if self.xfrac > 0:
            t = torch.randn([n, 2], device=dev) * self.xfrac_std
            t = choose(self.xfrac * self.p, t, torch.zeros_like(t), [n, 1])
            if dp is not None:
                t = torch.full_like(t, torch.erfinv(dp * 2 - 1) * self.xfrac_std)
            G = G @ translate2d_inv(t[:, 0] * w, t[:, 1] * h)
        if G is I_3:
            return images

        # Margins that keep the warped image inside the reflect-padded source.
        cx, cy = (w - 1) / 2, (h - 1) / 2
        corners = matrix([-cx, -cy, 1], [cx, -cy, 1], [cx, cy, 1], [-cx, cy, 1], device=dev)
        corners = G @ corners.t()
        hz_pad = self.Hz_geom.shape[0] // 4
        m = corners[:, :2, :].permute(1, 0, 2).flatten(1)
        m = torch.cat([-m, m]).max(dim=1).values
        m = m + misc.constant([hz_pad * 2 - cx, hz_pad * 2 - cy] * 2, device=dev)
        m = m.max(misc.constant([0, 0] * 2, device=dev))
        m = m.min(misc.constant([w - 1, h - 1] * 2, device=dev))
        mi = m.ceil().to(torch.int32)                     # (mx0, my0, mx1, my1), kept on the device
        mf = mi.float()
        mx0, my0, mx1, my1 = mf[0], mf[1], mf[2], mf[3]

        # Reflect pad into a static buffer (logical size h+my0+my1 x w+mx0+mx1 at its origin): no host
        # sync, so the step can be graph-captured (torch_utils/ops/reflect_pad.py).
        images = reflect_pad.reflect_pad_dyn(images, mi)
        G = translate2d((mx0 - mx1) / 2, (my0 - my1) / 2) @ G
        # extents (rows, cols) the up-sampling passes and their adjoints compute: the logical image plus
        # the filter reach (upfirdn2d.upsample2d_limited; the rest of the static buffer is never read)
        hd, wd = mi[1] + mi[3] + h, mi[0] + mi[2] + w
        lims = torch.stack([hd + 32, 2 * wd + 32, 2 * hd + 32, 2 * wd + 32,
                            2 * hd + 96, wd + 32, hd + 32, wd + 32]).to(torch.int32).reshape(4, 2)
        images = upfirdn2d.upsample2d_limited(images, self.Hz_geom, lims.unbind(0), up=2)
        G = scale2d(2, 2, device=dev) @ G @ scale2d_inv(2, 2, device=dev)
        G = translate2d(-0.5, -0.5, device=dev) @ G @ translate2d_inv(-0.5, -0.5, device=dev)
        shape = [n, c, (h + hz_pad * 2) * 2, (w + hz_pad * 2) * 2]
        dyn_h, dyn_w = (h + my0 + my1) * 2, (w + mx0 + mx1) * 2     # logical size of the upsampled image
        G = scale2d(2 / dyn_w, 2 / dyn_h) @ G @ scale2d_inv(2 / shape[3], 2 / shape[2], device=dev)
        dyn_hw = torch.stack([dyn_h, dyn_w]).to(torch.int32)
        # affine_grid + grid_sample (augment_mi.py:317-318) with the grid built inside the sampling kernel
        images = grid_sample_gradfix.affine_grid_sample(images, G[:, :2, :], shape, dyn_hw=dyn_hw)
        return upfirdn2d.downsample2d(x=images, f=self.Hz_geom, down=2, padding=-hz_pad * 2, flip_filter=True)

    # ------------------------------------------------------------------ colour
    def _color(self, images, dp):
        n, c, h, w = images.shape
        dev = images.device
        I_4 = torch.eye(4, device=dev)
        C = I_4
        if self.brightness > 0:
            b = torch.randn([n], device=dev) * self.brightness_std
            b = torch.where(torch.rand([n], device=dev) < self.brightness * self.p, b, torch.zeros_like(b))
            if dp is not None:
                b = torch.full_like(b, torch.erfinv(dp * 2 - 1) * self.brightness_std)
            C = translate3d(b, b, b) @ C
        if self.contrast > 0:
            k = torch.exp2(torch.randn([n], device=dev) * self.contrast_std)
            k = torch.where(torch.rand([n], device=dev) < self.contrast * self.p, k, torch.ones_like(k))
            if dp is not None:
                k = torch.full_like(k, torch.exp2(torch.erfinv(dp * 2 - 1) * self.contrast_std))
            C = scale3d(k, k, k) @ C
        v = misc.constant(np.asarray([1, 1, 1, 0]) / np.sqrt(3), device=dev)
        if self.lumaflip > 0:
            i = torch.floor(torch.rand([n, 1, 1], device=dev) * 2)
            i = torch.where(torch.rand([n, 1, 1], device=dev) < self.lumaflip * self.p, i, torch.zeros_like(i))
            if dp is not None:
                i = torch.full_like(i, torch.floor(dp * 2))
            C = (I_4 - 2 * v.ger(v) * i) @ C
        if self.hue > 0 and c > 1:
            th = (torch.rand([n], device=dev) * 2 - 1) * np.pi * self.hue_max
            th = torch.where(torch.rand([n], device=dev) < self.hue * self.p, th, torch.zeros_like(th))
            if dp is not None:
                th = torch.full_like(th, (dp * 2 - 1) * np.pi * self.hue_max)
            C = rotate3d(v, th) @ C
        if self.saturation > 0 and c > 1:
            s = torch.exp2(torch.randn([n, 1, 1], device=dev) * self.saturation_std)
            s = torch.where(torch.rand([n, 1, 1], device=dev) < self.saturation * self.p, s, torch.ones_like(s))
            if dp is not None:
                s = torch.full_like(s, torch.exp2(torch.erfinv(dp * 2 - 1) * self.saturation_std))
            C = (v.ger(v) + (I_4 - v.ger(v)) * s) @ C
        if C is I_4:
            return images
        images = images.reshape([n, c, h * w])
        if c == 3:
            images = C[:, :3, :3] @ images + C[:, :3, 3:]
        elif c == 1:
            Cm = C[:, :3, :].mean(dim=1, keepdims=True)
            images = images * Cm[:, :, :3].sum(dim=2, keepdims=True) + Cm[:, :, 3:]
        else:
            raise ValueError('Image must be RGB (3 channels) or L (1 channel)')
        return images.reshape([n, c, h, w])

    # ------------------------------------------------------------------ filtering / corruption
    def _filter(self, images, dp):
        n, c, h, w = images.shape
        dev = images.device
        nb = self.Hz_fbank.shape[0]
        assert len(self.imgfilter_bands) == nb
        power = misc.constant(np.array([10, 1, 1, 1]) / 13, device=dev)
        g = torch.ones([n, nb], device=dev)
        for i, band in enumerate(self.imgfilter_bands):
            ti = torch.exp2(torch.randn([n], device=dev) * self.imgfilter_std)
            ti = torch.where(torch.rand([n], device=dev) < self.imgfilter * self.p * band, ti, torch.ones_like(ti))
            if dp is not None:
                ti = torch.full_like(ti, torch.exp2(torch.erfinv(dp * 2 - 1) * self.imgfilter_std)) if band > 0 \
                    else torch.ones_like(ti)
            t = torch.ones([n, nb], device=dev)
            t[:, i] = ti
            t = t / (power * t.square()).sum(dim=-1, keepdims=True).sqrt()
            g = g * t
        hz = (g @ self.Hz_fbank).unsqueeze(1).repeat([1, c, 1]).reshape([n * c, 1, -1])
        p = self.Hz_fbank.shape[1] // 2
        images = images.reshape([1, n * c, h, w])
        images = torch.nn.functional.pad(input=images, pad=[p, p, p, p], mode='reflect')
        images = conv2d_gradfix.conv2d(input=images, weight=hz.unsqueeze(2), groups=n * c)
        images = conv2d_gradfix.conv2d(input=images, weight=hz.unsqueeze(3), groups=n * c)
        return images.reshape([n, c, h, w])

    def forward(self, images, allow_aug_debug_print=False, debug_percentile=None):
        assert isinstance(images, torch.Tensor) and images.ndim == 4
        n, c, h, w = images.shape
        dev = images.device
        dp = None if debug_percentile is None else torch.as_tensor(debug_percentile, dtype=torch.float32, device=dev)
        images = self._geometric(images, dp)
        images = self._color(images, dp)
        if self.imgfilter > 0:
            images = self._filter(images, dp)
        if self.noise > 0:
            sigma = torch.randn([n, 1, 1, 1], device=dev).abs() * self.noise_std
            sigma = torch.where(torch.rand([n, 1, 1, 1], device=dev) < self.noise * self.p, sigma, torch.zeros_like(sigma))
            if dp is not None:
                sigma = torch.full_like(sigma, torch.erfinv(dp) * self.noise_std)
            images = images + torch.randn([n, c, h, w], device=dev) * sigma
        if self.cutout > 0:
            size = torch.full([n, 2, 1, 1, 1], self.cutout_size, device=dev)
            size = torch.where(torch.rand([n, 1, 1, 1, 1], device=dev) < self.cutout * self.p, size, torch.zeros_like(size))
            center = torch.rand([n, 2, 1, 1, 1], device=dev)
            if dp is not None:
                size = torch.full_like(size, self.cutout_size)
                center = torch.full_like(center, dp)
            cxs = torch.arange(w, device=dev).reshape([1, 1, 1, -1])
            cys = torch.arange(h, device=dev).reshape([1, 1, -1, 1])
            mx = ((cxs + 0.5) / w - center[:, 0]).abs() >= size[:, 0] / 2
            my = ((cys + 0.5) / h - center[:, 1]).abs() >= size[:, 1] / 2
            images = images * torch.logical_or(mx, my).to(torch.float32)
        return images
