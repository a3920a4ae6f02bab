"""Convolution fused with FIR up/downsampling, on the HIP conv + upfirdn2d kernels.

API and numerics of SG3/torch_utils/ops/conv2d_resample.py:46-141 (`conv2d_resample`).  All
padding is expressed once, in the upsampled frame, and then split between the convolution and the
FIR pass according to which of five execution plans applies:

  plan          when                      execution                                 reference
  'fir_conv'    1x1 kernel, down > 1      FIR+decimate, then 1x1 conv               :94-97
  'conv_fir'    1x1 kernel, up > 1        1x1 conv, then zero-insert+FIR            :100-103
  'strided'     k x k, down > 1           FIR (pad only), then stride-`down` conv   :106-109
  'transposed'  up > 1                    stride-`up` transposed conv, then FIR     :112-129
  'direct'      symmetric non-neg. pads   conv with padding                         :132-134
  'generic'     anything else             FIR-up, conv, FIR-down                    :137-141
"""
import torch

from . import conv2d_gradfix
from . import upfirdn2d
from .upfirdn2d import _parse_padding, _get_filter_size


def _conv(x, w, stride=1, padding=0, groups=1, transpose=False, flip_weight=True):
    """flip_weight=True: correlation (F.conv2d semantics); False: true convolution."""
    kh, kw = int(w.shape[2]), int(w.shape[3])
    if (kh > 1 or kw > 1) and not flip_weight:
        w = w.flip([2, 3])
    fn = conv2d_gradfix.conv_transpose2d if transpose else conv2d_gradfix.conv2d
    return fn(x, w, stride=stride, padding=padding, groups=groups)


def _frame_padding(padding, f, up, down):
    """Padding in the upsampled frame, widened so the FIR keeps the output aligned."""
    fw, fh = _get_filter_size(f)
    p = list(_parse_padding(padding))  # x0, x1, y0, y1
    for k, (taps, lo) in enumerate([(fw, True), (fw, False), (fh, True), (fh, False)]):
        if up > 1:
            p[k] += (taps + up - 1) // 2 if lo else (taps - up) // 2
        if down > 1:
            p[k] += (taps - down + 1) // 2 if lo else (taps - down) // 2
    return p


def conv2d_resample(x, w, f=None, up=1, down=1, padding=0, groups=1, flip_weight=True, flip_filter=False):
    assert isinstance(x, torch.Tensor) and x.ndim == 4
    assert isinstance(w, torch.Tensor) and w.ndim == 4 and w.dtype == x.dtype
    assert f is None or (isinstance(f, torch.Tensor) and f.ndim in [1, 2] and f.dtype == torch.float32)
    assert isinstance(up, int) and up >= 1 and isinstance(down, int) and down >= 1
    assert isinstance(groups, int) and groups >= 1
    cout, cin_g, kh, kw = [int(s) for s in w.shape]
    x0, x1, y0, y1 = _frame_padding(padding, f, up, down)
    pointwise = (kh == 1 and kw == 1)
    fir = upfirdn2d.upfirdn2d

    if pointwise and down > 1 and up == 1:
        t = fir(x, f, down=down, padding=[x0, x1, y0, y1], flip_filter=flip_filter)
        return _conv(t, w, groups=groups, flip_weight=flip_weight)

    if pointwise and up > 1 and down == 1:
        t = _conv(x, w, groups=groups, flip_weight=flip_weight)
        return fir(t, f, up=up, padding=[x0, x1, y0, y1], gain=up * up, flip_filter=flip_filter)

    if down > 1 and up == 1:
        t = fir(x, f, padding=[x0, x1, y0, y1], flip_filter=flip_filter)
        return _conv(t, w, stride=down, groups=groups, flip_weight=flip_weight)

    if up > 1:
        # transposed-conv weight layout [Cin, Cout/groups, kh, kw]
        if groups == 1:
            wt = w.transpose(0, 1)
        else:
            wt = w.reshape(groups, cout // groups, cin_g, kh, kw).transpose(1, 2)
            wt = wt.reshape(groups * cin_g, cout // groups, kh, kw)
        x0, x1 = x0 - (kw - 1), x1 - (kw - up)
        y0, y1 = y0 - (kh - 1), y1 - (kh - up)
        # the part of the padding both sides share is cropped by the transposed conv itself
        cx = max(-max(x0, x1), 0)
        cy = max(-max(y0, y1), 0)
        t = _conv(x, wt, stride=up, padding=[cy, cx], groups=groups, transpose=True, flip_weight=not flip_weight)
        t = fir(t, f, padding=[x0 + cx, x1 + cx, y0 + cy, y1 + cy], gain=up * up, flip_filter=flip_filter)
        if down > 1:
            t = fir(t, f, down=down, flip_filter=flip_filter)
        return t

    if up == 1 and down == 1 and x0 == x1 and y0 == y1 and min(x0, y0) >= 0:
        return _conv(x, w, padding=[y0, x0], groups=groups, flip_weight=flip_weight)

    t = fir(x, f if up > 1 else None, up=up, padding=[x0, x1, y0, y1], gain=up * up, flip_filter=flip_filter)
    t = _conv(t, w, groups=groups, flip_weight=flip_weight)
    if down > 1:
        t = fir(t, f, down=down, flip_filter=flip_filter)
    return t
