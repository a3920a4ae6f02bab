"""2-D convolution / transposed convolution on MI355X MFMA (HIP kernels sg2_conv2d, sg2_conv2d_wgrad)
with gradients of arbitrary order.

Drop-in for SG3/torch_utils/ops/conv2d_gradfix.py (:37-45 `conv2d`, `conv_transpose2d`,
`no_weight_gradients`, module flags `enabled` / `weight_gradients_disabled`).  The reference
routes to cuDNN (its custom op is disabled on torch >= 1.11, :53-55); here every call runs the HIP
implicit-GEMM kernels, and the three ops {conv, transposed conv, weight gradient} are closed under
differentiation, so the path-length (G) and R1 (D) double-backward passes stay on MFMA:

    conv2d(x, w)        : dx = conv_transpose2d(dy, w)   dw = wgrad(dy, x)
    conv_transpose2d(x,w): dx = conv2d(dy, w)            dw = wgrad(x, dy)   (roles swapped)
    wgrad(g, x) -> dw   : dg = conv2d(x, ddw)            dx = conv_transpose2d(g, ddw)

Activations are NHWC in memory (torch channels_last); weights are packed K-contiguous per output
channel before each launch (a few MB at most).
"""
import contextlib
import ctypes
import os

import numpy as np
import torch

import sg2hip as _hip

enabled = True                      # accepted for API compatibility; the HIP path is always used
weight_gradients_disabled = False   # skip dw (reference :21-33); values are unaffected


@contextlib.contextmanager
def no_weight_gradients(disable=True):
    global weight_gradients_disabled
    old = weight_gradients_disabled
    if disable:
        weight_gradients_disabled = True
    yield
    weight_gradients_disabled = old


def _pair(v):
    if isinstance(v, (list, tuple)):
        assert len(v) == 2
        return int(v[0]), int(v[1])
    return int(v), int(v)


_CL = torch.channels_last


def _nhwc(t):
    t = t.contiguous(memory_format=_CL)
    if t.data_ptr() % 16:
        t = t.clone(memory_format=_CL)
    return t


# f32 convolutions (the 4^2..16^2 blocks) on pre-split operands: each f32 operand is split ONCE per call into its
# three bf16 planes (sg2_split3, with the layer's modulation folded in) and the kernels stage the planes directly
# (SG2_F32S3) instead of every workgroup re-splitting its tiles inside the K loop.  NOT bitwise the same arithmetic
# as the in-loop split (the two forms tile and order their sums differently): what is held is accuracy,
# within 2e-6 of float64 and within 1.5x of the in-loop split's error
# (tests/test_ops_gpu.py::test_presplit_f32_accuracy).  SG2_P3=0 keeps the in-loop split (A/B switch).
presplit = os.environ.get('SG2_P3', '1') != '0' and os.environ.get('SG2_F32_EXACT', '0') != '1'
# the forward / input-gradient convolutions measured no faster on pre-split operands (tools/f32_ab.py: 16^2 bs64
# 0.484 -> 0.430 ms with the split included, 8^2 and 4^2 0.082 -> 0.085 / 0.044 -> 0.055): the weight gradients
# alone take them (0.611 -> 0.488, 0.312 -> 0.257, 0.124 -> 0.111 ms)
presplit_fwd = os.environ.get('SG2_P3_FWD', '0') != '0'


def split3(x, scale=None, packed=False):
    """f32 activation [N, C, H, W] (NHWC memory), or (packed) a packed weight [.., C] in its memory order ->
    [3, numel] bf16 planes of x * scale[n, c]."""
    C = x.shape[-1] if packed else x.shape[1]
    per = 1 if packed else x.shape[2] * x.shape[3]
    planes = torch.empty([3, x.numel()], dtype=torch.bfloat16, device=x.device)
    sc = scale.float().contiguous() if scale is not None else None
    _hip.check(_hip.lib().sg2_split3(_hip.ptr(planes), _hip.ptr(x), x.numel(), C, per, _hip.ptr(sc),
                                     _hip.stream_ptr(x.device)), 'sg2_split3')
    return planes


def _split_w(wp):
    """The planes of a packed f32 weight, cached with the pack inside a pack_cache() scope."""
    key = ('s3', wp.data_ptr(), wp._version, tuple(wp.shape))
    if _pack_cache is not None:
        hit = _pack_cache.get(key)
        if hit is not None:
            return hit[0]
    out = split3(wp.contiguous(), packed=True)
    if _pack_cache is not None:
        _pack_cache[key] = (out, wp)
    return out


def _p3(x, cin):
    return presplit and x.dtype == torch.float32 and cin % 8 == 0 and x.is_cuda


_WS_LIMIT = 1 << 23  # split-K f32 workspace only for small outputs (low-resolution layers)
_CLEAN_WS = {}       # device -> persistent zeroed split-K workspace (every call leaves it zeroed)


_PERSIST_WS = os.environ.get('SG2_CLEAN_WS', '1') != '0'   # A/B switch: 0 = a fresh zeroed workspace per call


def _workspace(x, total):
    """(workspace, clean): the device's persistent zeroed workspace when it can be used (created outside any
    graph capture, so eager calls and replayed graphs share one buffer), else a fresh one per call."""
    if total > _WS_LIMIT:
        return None, False
    if not _PERSIST_WS:
        return torch.zeros([total], dtype=torch.float32, device=x.device), False
    ws = _CLEAN_WS.get(x.device)
    if ws is None:
        if torch.cuda.is_current_stream_capturing():
            return torch.empty([total], dtype=torch.float32, device=x.device), False
        ws = _CLEAN_WS[x.device] = torch.zeros([_WS_LIMIT], dtype=torch.float32, device=x.device)
    return ws, True


@contextlib.contextmanager
def _split_k(x, clean):
    """Split-K calls on the persistent workspace: the call takes it as zeroed and leaves it zeroed (its
    finalize clears what it read).  A call that fails (a launch error, an aborted capture) may leave it dirty
    and every later split-K conv would add that garbage: drop the buffer then, so the next call allocates a
    fresh zeroed one."""
    try:
        with _hip.clean_workspace(clean):
            yield
    except BaseException:
        if clean:
            _CLEAN_WS.pop(x.device, None)
        raise


up2_min = int(os.environ.get('SG2_UP2_MIN', '16'))   # smallest input edge the up-2 kernel takes (edge split on)


def _up2_ok(x, cout, oh, ow, kh, kw, stride, pad, transpose):
    """sg2_conv3x3_up2 serves the 16-bit stride-2 transposed 3x3 convs with padding 0 (output 2H+1).  Its 16 x 8
    cell tiles cover the (H+1) x (W+1) cells raggedly (15 tiles for 33 x 33 cells at 32^2); with H % 8 == W % 16
    == 0 the kernel splits off the last cell row and column as three-tap strips (8 + 2/3 tile-equivalents at 32^2),
    which is what lets it take the 16^2 and 32^2 inputs from the four-phase implicit GEMM (tools/up2_ab.py).
    Unsplit (ragged) shapes take it from 64^2 up: 128^2 -> 257^2 C 128 -> 64: 0.168 vs 0.264 ms; 64^2 C 256 -> 128:
    0.152 vs 0.181 ms; 32^2 C 512 -> 256: 0.163 vs 0.143 ms ragged."""
    n, cin, h, w = x.shape
    if not (transpose and stride == 2 and kh == 3 and kw == 3 and tuple(pad) == (0, 0) and oh == 2 * h + 1 and
            ow == 2 * w + 1 and x.dtype in (torch.float16, torch.bfloat16) and cin % 32 == 0 and cout % 8 == 0):
        return False
    if h >= 64 and w >= 64:
        return True
    split = h % 8 == 0 and w % 16 == 0 and os.environ.get('SG2_UP2_EDGE', '1') != '0'
    return split and h >= up2_min and w >= up2_min


def _conv_up2(x, wp, cout, in_scale=None):
    n, cin, h, w = x.shape
    y = torch.empty([n, cout, 2 * h + 1, 2 * w + 1], dtype=x.dtype, device=x.device, memory_format=_CL)
    _hip.check(_hip.lib().sg2_conv3x3_up2(
        _hip.ptr(y), _hip.ptr(x), _hip.ptr(wp), _hip.dtype_code(x), n, cin, h, w, cout, _hip.ptr(in_scale),
        _hip.stream_ptr(x.device)), 'sg2_conv3x3_up2')
    return y


def _conv_raw(x, wp, cout, oh, ow, kh, kw, stride, pad, transpose):
    """x [N,Cin,H,W] (NHWC memory), wp packed [Cout][kh][kw][Cin] -> y [N,Cout,oh,ow] (NHWC memory)."""
    if _up2_ok(x, cout, oh, ow, kh, kw, stride, pad, transpose):
        return _conv_up2(x, wp, cout)
    n, cin, h, w = x.shape
    y = torch.empty([n, cout, oh, ow], dtype=x.dtype, device=x.device, memory_format=_CL)
    total = n * cout * oh * ow
    ws, clean = _workspace(x, total)
    xa, wa, dt = x, wp, _hip.dtype_code(x)
    if presplit_fwd and _p3(x, cin):
        xa, wa, dt = split3(_nhwc(x)), _split_w(wp), _hip.F32S3
    with _split_k(x, clean):
        _hip.check(_hip.lib().sg2_conv2d(
            _hip.ptr(y), _hip.ptr(xa), _hip.ptr(wa), dt, n, cin, h, w, cout, oh, ow, kh, kw,
            stride, pad[0], pad[1], int(transpose), _hip.ptr(ws), ws.numel() if ws is not None else 0,
            _hip.stream_ptr(x.device)), 'sg2_conv2d')
    return y


def conv_fused(x, wp, cout, oh, ow, kh, kw, stride, pad, transpose=False, in_scale=None, out_scale=None,
               noise=None, noise_gain=1.0, bias=None, act=0, alpha=0.2, gain=1.0, clamp=-1.0, residual=None,
               aux_mode=0, dot_src=None, dot_out=None):
    """sg2_conv2d_fused: y = round(clamp(act(conv(x * in_scale, w) * out_scale + noise * g + bias) * gain))
    + residual.  Returns (y, aux) with aux = conv result (aux_mode 1) or activation (aux_mode 2); with
    dot_src also dot[n, o] = sum_p conv(...)[n, o, p] * dot_src[n, o, p] -> (y, aux, dot).  dot_out: a
    zeroed f32 [N, Cout] buffer for dot (the call then skips its own memset)."""
    if (out_scale is None and noise is None and bias is None and residual is None and dot_src is None and act == 0 and
            gain == 1.0 and clamp < 0 and not aux_mode and _up2_ok(x, cout, oh, ow, kh, kw, stride, pad, transpose)):
        return _conv_up2(x, wp, cout, in_scale), None
    n, cin, h, w = x.shape
    y = torch.empty([n, cout, oh, ow], dtype=x.dtype, device=x.device, memory_format=_CL)
    aux = torch.empty_like(y) if aux_mode else None
    if residual is not None:
        residual = _nhwc(residual)
        assert residual.shape == y.shape and residual.dtype == y.dtype
    dot = None
    if dot_src is not None:
        dot_src = _nhwc(dot_src)
        assert dot_src.shape == y.shape and dot_src.dtype == y.dtype
        dot = dot_out if dot_out is not None else torch.empty([n, cout], dtype=torch.float32, device=x.device)
    epi = None
    if any(v is not None for v in (out_scale, noise, bias, residual, dot_src)) or act != 0 or gain != 1.0 or \
            clamp >= 0 or aux_mode:
        epi = _hip.Epilogue(_hip.ptr(out_scale), _hip.ptr(noise), _hip.ptr(bias), _hip.ptr(residual), _hip.ptr(aux),
                            float(noise_gain), float(alpha), float(gain), float(clamp), int(act), int(aux_mode),
                            _hip.ptr(dot_src), _hip.ptr(dot))
    total = n * cout * oh * ow
    ws, clean = _workspace(x, total)
    xa, wa, dt, isc = x, wp, _hip.dtype_code(x), in_scale
    if presplit_fwd and _p3(x, cin):
        xa, wa, dt, isc = split3(_nhwc(x), in_scale), _split_w(wp), _hip.F32S3, None
    with _hip.zeroed_accumulators(dot_out is not None and dot is not None), _split_k(x, clean):
        _hip.check(_hip.lib().sg2_conv2d_fused(
            _hip.ptr(y), _hip.ptr(xa), _hip.ptr(wa), dt, n, cin, h, w, cout, oh, ow, kh, kw,
            stride, pad[0], pad[1], int(transpose), _hip.ptr(isc), ctypes.byref(epi) if epi is not None else None,
            _hip.ptr(ws), ws.numel() if ws is not None else 0, _hip.stream_ptr(x.device)), 'sg2_conv2d_fused')
    return (y, aux, dot) if dot_src is not None else (y, aux)


def _wgrad_raw(g, x, kh, kw, stride, pad, x_scale=None, g_scale=None, alpha=1.0, out=None, param_layout=False):
    """dw[a, b, ky, kx] = alpha * sum g[n,a,oy,ox] (* g_scale[n,a]) x[n,b,oy*s+ky-p,ox*s+kx-p] (* x_scale[n,b]);
    returns f32 [A,B,kh,kw] (NHWC-packed: a permuted view).  alpha: a layer's weight gain (the backward of w * gain).
    out: a zeroed f32 buffer of A*kh*kw*B elements to accumulate into (the call skips its memset).
    param_layout: where the library can (f32 layers under the deterministic reductions, sg2_conv2d_wgrad_oikk),
    write dw contiguous in [A, B, kh, kw] -- the parameter's own layout, which autograd's gradient accumulation then
    takes as is instead of copying a permuted view; 'swap': contiguous [B, A, kh, kw], returned as its [A, B, kh, kw]
    view (a transposed conv's weight gradient, whose caller transposes A and B back)."""
    n, a, oh, ow = g.shape
    _, b, h, w = x.shape
    ga, xa, dt, gs, xs = g, x, _hip.dtype_code(g), g_scale, x_scale
    if _p3(g, 8) and a % 8 == 0 and b % 8 == 0 and not (kh == 1 and kw == 1 and min(a, b) <= 4):
        ga, xa, dt, gs, xs = split3(_nhwc(g), g_scale), split3(_nhwc(x), x_scale), _hip.F32S3, None, None
        if param_layout and _hip.det_active() and b % 4 == 0 and kh * kw <= 9:
            swap = param_layout == 'swap'
            shape = [b, a, kh, kw] if swap else [a, b, kh, kw]
            dw = out.view(*shape) if out is not None else torch.empty(shape, dtype=torch.float32, device=g.device)
            with _hip.zeroed_accumulators(out is not None):
                _hip.check(_hip.lib().sg2_conv2d_wgrad_oikk(
                    _hip.ptr(dw), _hip.ptr(ga), _hip.ptr(xa), dt, n, a, oh, ow, b, h, w, kh, kw, stride,
                    pad[0], pad[1], float(alpha), int(swap), _hip.stream_ptr(g.device)), 'sg2_conv2d_wgrad_oikk')
            return dw.transpose(0, 1) if swap else dw
    dw = out.view(a, kh, kw, b) if out is not None else torch.empty([a, kh, kw, b], dtype=torch.float32, device=g.device)
    with _hip.zeroed_accumulators(out is not None):
        _hip.check(_hip.lib().sg2_conv2d_wgrad(
            _hip.ptr(dw), _hip.ptr(ga), _hip.ptr(xa), dt, n, a, oh, ow, b, h, w, kh, kw, stride,
            pad[0], pad[1], _hip.ptr(gs), _hip.ptr(xs), float(alpha), _hip.stream_ptr(g.device)),
            'sg2_conv2d_wgrad')
    return dw.permute(0, 3, 1, 2)


_pack_cache = None   # {key: packed} while a pack_cache() scope is open
_pack_record = None  # the entries of the plan being recorded (pack_cache(plan=...) without a plan yet)
prepack_enabled = os.environ.get('SG2_PREPACK', '1') != '0'


class _PackPlan:
    """Every parameter pack a training phase makes, done at the phase start in ONE sg2_pack_weight_multi launch
    into persistent buffers (bitwise the per-call sg2_pack_weight results), which the phase's pack requests then
    find in the cache: ~40 launches per phase (158 per step) become one per 64 packs.  Recorded from the phase's
    first run; the buffers and the source addresses are fixed and the table travels in the kernel arguments, so the
    launch can be captured into the phase's HIP graph and replayed after every optimiser step."""

    DESC = np.dtype([('out', '<u8'), ('in', '<u8'), ('sa', '<i8'), ('sb', '<i8'), ('sk', '<i8'), ('out_dtype', '<i4'),
                     ('in_dtype', '<i4'), ('A', '<i4'), ('B', '<i4'), ('K', '<i4'), ('flip', '<i4'), ('scale', '<f4'),
                     ('block0', '<i4')])   # include/sg2hip.h sg2_pack_desc (72 bytes)

    def __init__(self, entries):
        self.entries = entries                   # (base param, storage offset, shape, stride, a_dim, dtype, flip, scale)
        self.outs, rows = [], []
        for base, off, shape, stride, a_dim, dtype, flip, scale in entries:
            b_dim = 1 - a_dim
            A, B, kh, kw = shape[a_dim], shape[b_dim], shape[2], shape[3]
            out = torch.empty([A, kh, kw, B], dtype=dtype or base.dtype, device=base.device)
            self.outs.append(out)
            rows.append((out.data_ptr(), self._addr(base, off), stride[a_dim], stride[b_dim],
                         stride[3], _hip._DTYPES[out.dtype], _hip._DTYPES[base.dtype], A, B, kh * kw, int(flip),
                         float(scale), 0))                 # (block0: set by the library)
        self.table = np.array(rows, dtype=self.DESC)   # host table: the library copies it into the launch arguments
        self.src = [e[0].data_ptr() for e in entries]

    @staticmethod
    def _addr(base, off):
        return base.untyped_storage().data_ptr() + off * base.element_size()

    def valid(self):
        return all(e[0].data_ptr() == p for e, p in zip(self.entries, self.src))

    def run(self, cache):
        dev = self.entries[0][0].device
        _hip.check(_hip.lib().sg2_pack_weight_multi(self.table.ctypes.data, len(self.entries), _hip.stream_ptr(dev)),
                   'sg2_pack_weight_multi')
        for (base, off, shape, stride, a_dim, dtype, flip, scale), out in zip(self.entries, self.outs):
            key = (self._addr(base, off), base._version, shape, stride, a_dim, dtype, bool(flip), float(scale))
            cache[key] = (out, base)


@contextlib.contextmanager
def pack_cache(plan=None):
    """Reuse weight packs inside the scope: a training phase packs every conv weight of D twice per form
    (the fake and the real pass of Dmain, their backward), with the parameters unchanged in between.  Only
    packs of parameters (or views of them) are cached, keyed by storage, version, view geometry and the
    pack form; the trainer opens one scope per phase (eagerly or while capturing the phase's graph), so
    the optimizer step never runs inside one.  plan: a dict owned by the caller (the trainer's phase) that holds
    the scope's pack set under 'pack_plan': its first scope records the packs, later scopes make them all up front
    in one launch (_PackPlan)."""
    global _pack_cache, _pack_record
    prev, prev_rec = _pack_cache, _pack_record
    _pack_cache = {} if prev is None else prev
    recording = None
    if plan is not None and prev is None and prepack_enabled:
        pl = plan.get('pack_plan')
        if pl is not None and not pl.valid():
            pl = plan['pack_plan'] = None
        if pl is not None:
            pl.run(_pack_cache)
        else:
            recording = _pack_record = []
    try:
        yield
    finally:
        _pack_cache = prev
        _pack_record = prev_rec
        if recording and all(e[0].is_cuda for e in recording):
            plan['pack_plan'] = _PackPlan(recording)


def _pack(w, a_dim, dtype, flip, scale=1.0):
    """out[a][ky][kx][b] = scale * w[.., ky', kx'] with (a, b) = dims (a_dim, 1 - a_dim) of w, cast to dtype,
    the taps reversed when flip -- one sg2_pack_weight launch instead of a strided copy (and, with scale, of
    the reference's `weight * weight_gain` multiply)."""
    key = None
    if _pack_cache is not None and (isinstance(w, torch.nn.Parameter) or isinstance(w._base, torch.nn.Parameter)):
        base = w if isinstance(w, torch.nn.Parameter) else w._base
        key = (w.data_ptr(), base._version, tuple(w.shape), tuple(w.stride()), a_dim, dtype, bool(flip), float(scale))
        hit = _pack_cache.get(key)
        if hit is not None:
            return hit[0]
    out = _pack_raw(w, a_dim, dtype, flip, scale)
    if key is not None:
        _pack_cache[key] = (out, w)    # (w keeps the parameter view alive for the scope)
        if _pack_record is not None and w.dim() == 4 and w.shape[2] * w.shape[3] <= 9 and \
                w.stride(2) == w.shape[3] * w.stride(3):
            _pack_record.append((base, w.storage_offset(), tuple(w.shape), tuple(w.stride()), a_dim, dtype,
                                 bool(flip), float(scale)))
    return out


def _pack_raw(w, a_dim, dtype, flip, scale):
    b_dim = 1 - a_dim
    A, B, kh, kw = w.shape[a_dim], w.shape[b_dim], w.shape[2], w.shape[3]
    if kh * kw > 9:    # no such conv in the networks; layout copy on the device
        w = w.flip([2, 3]) if flip else w
        w = w * scale if scale != 1.0 else w
        return w.permute(a_dim, 2, 3, b_dim).to(dtype or w.dtype, memory_format=torch.contiguous_format)
    if w.stride(2) != kw * w.stride(3):
        w = w.contiguous()
    out = torch.empty([A, kh, kw, B], dtype=dtype or w.dtype, device=w.device)
    _hip.require_device(w)
    _hip.check(_hip.lib().sg2_pack_weight(
        _hip.ptr(out), _hip.dtype_code(out), _hip.ptr(w), _hip.dtype_code(w), A, B, kh * kw, w.stride(a_dim),
        w.stride(b_dim), w.stride(3), 1 if flip else 0, float(scale), _hip.stream_ptr(w.device)), 'sg2_pack_weight')
    return out


def _pack_conv(w, dtype=None, flip=False, scale=1.0):   # [O, I, kh, kw] -> [O][kh][kw][I], cast (and scaled) in one pass
    return _pack(w, 0, dtype, flip, scale)


def _pack_convT(w, dtype=None, flip=False, scale=1.0):  # [I, O, kh, kw] -> [O][kh][kw][I]
    return _pack(w, 1, dtype, flip, scale)


def _halo_ok(x, kh, kw, stride, pad, out_hw):
    """The LDS-halo 3x3 kernel (sg2_conv3x3) serves 16-bit 3x3/s1/p1 layers of the 16^2+ blocks."""
    n, c, h, w = x.shape
    return (kh == 3 and kw == 3 and stride == 1 and tuple(pad) == (1, 1) and tuple(out_hw) == (h, w) and
            x.dtype in (torch.float16, torch.bfloat16) and c % 8 == 0 and h >= 16 and w >= 16)


def _halo_s2_ok(x, kh, kw, stride, pad, dot=False, cout=None, scaled=False):
    """The stride-2 / pad-0 forms of sg2_conv3x3_s2 for 16-bit 3x3 layers.  The 32x4 halo tile, measured against
    the implicit GEMM (tools/s2_ab.py, profiles/r02_s2_ab.log), wins for outputs <= 16 wide in every form (the
    discriminator's 32^2 / 16^2 down layers), and in the out_scale + dot form (the up layers' input gradient,
    where the implicit GEMM's dot epilogue is slow) also for inputs of <= 128 channels.  The wide down layers
    (outputs >= 32 wide, Cin % 32 == 0, Cout % 128 == 0, no modulation / noise / dot: the D blocks' conv1, given
    `cout`) take the LDS-DMA implicit GEMM of the same entry point (conv3x3.hip conv3x3_s2g_kernel,
    tools/s2g_ab.py); other wide shapes stay on the generic implicit GEMM."""
    n, c, h, w = x.shape
    p = tuple(pad) if isinstance(pad, (tuple, list)) else (pad, pad)
    if not (kh == 3 and kw == 3 and stride == 2 and p == (0, 0) and x.dtype in (torch.float16, torch.bfloat16) and
            c % 8 == 0 and h >= 17 and w >= 17):
        return False
    ow = (w - 3) // 2 + 1
    if cout is not None and not dot and not scaled and c % 32 == 0 and cout % 128 == 0 and ow >= 32:
        return True
    return ow <= 16 or (dot and c <= 128)


def conv3x3_fused(x, wp, cout, in_scale=None, out_scale=None, noise=None, noise_gain=0.0, bias=None, act=0,
                  alpha=0.2, gain=1.0, clamp=-1.0, want_raw=False, dot_src=None, stride=1, residual=None,
                  raw_act=False, dot_out=None):
    """sg2_conv3x3 (stride 1, pad 1) / sg2_conv3x3_s2 (stride 2, pad 0) launch.  x NHWC 16-bit, wp packed
    [Cout][3][3][Cin].  Returns (y, raw or None, dot or None) with dot[n,o] = sum_p conv(x)[n,o,p] *
    dot_src[n,o,p]; with stride 2 an optional residual is added after the epilogue and raw_act makes raw
    the pre-residual epilogue value."""
    n, cin, h, w = x.shape
    oh, ow = (h, w) if stride == 1 else ((h - 3) // 2 + 1, (w - 3) // 2 + 1)
    y = torch.empty([n, cout, oh, ow], dtype=x.dtype, device=x.device, memory_format=_CL)
    raw = torch.empty_like(y) if want_raw else None
    dot = None
    if dot_src is not None:
        dot_src = _nhwc(dot_src)
        assert dot_src.shape == y.shape and dot_src.dtype == y.dtype
        dot = dot_out if dot_out is not None else torch.empty([n, cout], dtype=torch.float32, device=x.device)
    lib = _hip.lib()
    zeroed = dot_out is not None and dot is not None   # the caller zeroed dot_out (no memset in the call)
    common = (_hip.ptr(y), _hip.ptr(raw), _hip.ptr(x), _hip.ptr(wp), _hip.dtype_code(x), n, cin, h, w, cout,
              _hip.ptr(in_scale), _hip.ptr(out_scale), _hip.ptr(noise), float(noise_gain), _hip.ptr(bias), int(act),
              float(alpha), float(gain), float(clamp))
    if stride == 1:
        assert residual is None
        with _hip.zeroed_accumulators(zeroed):
            _hip.check(lib.sg2_conv3x3(*common, _hip.ptr(dot_src), _hip.ptr(dot), _hip.stream_ptr(x.device)),
                       'sg2_conv3x3')
    else:
        assert stride == 2
        if residual is not None:
            residual = _nhwc(residual)
            assert residual.shape == y.shape and residual.dtype == y.dtype
        with _hip.zeroed_accumulators(zeroed):
            _hip.check(lib.sg2_conv3x3_s2(*common, _hip.ptr(residual), int(bool(raw_act)), _hip.ptr(dot_src),
                                          _hip.ptr(dot), _hip.stream_ptr(x.device)), 'sg2_conv3x3_s2')
    return (y, raw, dot) if dot_src is not None else (y, raw)


def layer_bwd(dy, y, c=None, d=None, act=1, alpha=0.2, gain=1.0, clamp=-1.0, want_db=True, want_dd=True,
              want_dnoise=True, acc=None):
    """sg2_layer_bwd: returns (dc, db[C] or None, dd[N,C] or None, dnoise[N,1,H,W] or None).  acc: a zeroed
    f32 buffer of (C if want_db) + (N*C if want_dd) elements holding db then dd (no memset in the call)."""
    y = _nhwc(y)
    dy = _nhwc(dy)
    n, ch, h, w = y.shape
    dc = torch.empty_like(y)
    f32 = dict(dtype=torch.float32, device=y.device)
    want_dd = want_dd and d is not None
    if acc is not None:
        db = acc[:ch] if want_db else None
        dd = acc[(ch if want_db else 0):][:n * ch].view(n, ch) if want_dd else None
    elif want_db and want_dd:   # one buffer: the library zeroes both accumulators with one memset
        buf = torch.empty([ch + n * ch], **f32)
        db, dd = buf[:ch], buf[ch:].view(n, ch)
    else:
        db = torch.empty([ch], **f32) if want_db else None
        dd = torch.empty([n, ch], **f32) if want_dd else None
    dn = torch.empty([n, 1, h, w], **f32) if want_dnoise else None
    c = _nhwc(c) if c is not None else None
    with _hip.zeroed_accumulators(acc is not None):
        _hip.check(_hip.lib().sg2_layer_bwd(
            _hip.ptr(dc), _hip.ptr(db), _hip.ptr(dd), _hip.ptr(dn), _hip.ptr(dy), _hip.ptr(y), _hip.ptr(c),
            _hip.ptr(d), _hip.dtype_code(y), n, h * w, ch, int(act), float(alpha), float(gain), float(clamp),
            _hip.stream_ptr(y.device)), 'sg2_layer_bwd')
    return dc, db, dd, dn


def vjp_axpy(a, sa=None, b=None, sb=None, y=None, act=0, alpha=0.2, gain=1.0, clamp=-1.0, e=None):
    """sg2_vjp_axpy: out = act'(a * sa[n,c] + b * sb[n,c]; y) (act' only with y) and, with e, dot[n,c] =
    sum_p a * e (f32).  a, b, y, e: [N, C, H, W] of one dtype (NHWC memory); sa / sb: [N, C] float or None.
    Returns (out, dot or None).  Channel counts that are not a multiple of 8 (toRGB's output side) take
    the same arithmetic as torch ops (f32, one rounding)."""
    n, ch, h, w = a.shape
    _hip.require_device(a)
    if ch % 8:
        v = a.float() * (sa.float()[:, :, None, None] if sa is not None else 1.0)
        if b is not None:
            v = v + b.float() * (sb.float()[:, :, None, None] if sb is not None else 1.0)
        if y is not None:
            yf = y.float()
            v = v * gain
            if act == 1:
                v = torch.where(yf > 0, v, v * alpha)
            if clamp >= 0:
                v = torch.where((yf > -clamp) & (yf < clamp), v, torch.zeros_like(v))
        dot = (a.float() * e.float()).sum([2, 3]) if e is not None else None
        return _nhwc(v.to(a.dtype)), dot
    a = _nhwc(a)
    args = [_nhwc(t) if t is not None else None for t in (b, y, e)]
    for t in args:
        assert t is None or (t.shape == a.shape and t.dtype == a.dtype), 'vjp_axpy: operand shape / dtype'
    b, y, e = args
    sa = sa.float().contiguous() if sa is not None else None
    sb = sb.float().contiguous() if sb is not None else None
    out = torch.empty_like(a)
    dot = torch.empty([n, ch], dtype=torch.float32, device=a.device) if e is not None else None
    _hip.check(_hip.lib().sg2_vjp_axpy(
        _hip.ptr(out), _hip.ptr(a), _hip.ptr(sa), _hip.ptr(b), _hip.ptr(sb), _hip.ptr(y), int(act), float(alpha),
        float(gain), float(clamp), _hip.ptr(e), _hip.ptr(dot), _hip.dtype_code(a), n, h * w, ch,
        _hip.stream_ptr(a.device)), 'sg2_vjp_axpy')
    return out, dot


class _DotHW(torch.autograd.Function):
    """out[n, c] = sum_{h,w} round(a * b) in f32 (sg2_dot_hw): (a * b).sum([2, 3], dtype=float32) without
    the full-size product in HBM.  The backward is composed of differentiable ops (double backward)."""

    @staticmethod
    def forward(ctx, a, b):
        a, b = _nhwc(a), _nhwc(b)
        n, c, h, w = a.shape
        out = torch.empty([n, c], dtype=torch.float32, device=a.device)
        _hip.check(_hip.lib().sg2_dot_hw(_hip.ptr(out), _hip.ptr(a), _hip.ptr(b), _hip.dtype_code(a), n, h * w, c,
                                         _hip.stream_ptr(a.device)), 'sg2_dot_hw')
        ctx.save_for_backward(a, b)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g_ = g.to(a.dtype)[:, :, None, None]
        return (g_ * b if ctx.needs_input_grad[0] else None), (g_ * a if ctx.needs_input_grad[1] else None)


def dot_hw(a, b):
    """(a * b).sum([2, 3], dtype=float32) for 16-bit [N, C, H, W] tensors (C % 8 == 0) on the HIP kernel."""
    if a.dtype in (torch.float16, torch.bfloat16) and b.dtype == a.dtype and a.shape == b.shape and \
            a.shape[1] % 8 == 0 and a.is_cuda:
        return _DotHW.apply(a, b)
    return (a * b).sum([2, 3], dtype=torch.float32)


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad, out_hw):
        x = _nhwc(x)
        o, i, kh, kw = w.shape
        assert x.shape[1] == i and x.dtype == w.dtype
        oh, ow = out_hw
        if _halo_ok(x, kh, kw, stride, pad, out_hw):
            y = conv3x3_fused(x, _pack_conv(w), o)[0]
        elif _halo_s2_ok(x, kh, kw, stride, pad, cout=o):
            y = conv3x3_fused(x, _pack_conv(w), o, stride=2)[0]
        else:
            y = _conv_raw(x, _pack_conv(w), o, oh, ow, kh, kw, stride, pad, False)
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.pad = stride, pad
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = _ConvT2d.apply(dy, w, ctx.stride, ctx.pad, tuple(x.shape[2:]))
        if ctx.needs_input_grad[1] and not weight_gradients_disabled:
            dw = _WGrad.apply(dy, x, tuple(w.shape[2:]), ctx.stride, ctx.pad).to(w.dtype)
        return dx, dw, None, None, None


class _ConvT2d(torch.autograd.Function):
    """y = conv_transpose2d(x, w[I, O, kh, kw], stride, padding) with explicit output size."""

    @staticmethod
    def forward(ctx, x, w, stride, pad, out_hw):
        x = _nhwc(x)
        i, o, kh, kw = w.shape
        assert x.shape[1] == i and x.dtype == w.dtype
        oh, ow = out_hw
        if _halo_ok(x, kh, kw, stride, pad, out_hw):
            # stride-1 transposed conv == correlation with the spatially flipped, transposed kernel
            y = conv3x3_fused(x, _pack_convT(w, flip=True), o)[0]
        else:
            y = _conv_raw(x, _pack_convT(w), o, oh, ow, kh, kw, stride, pad, True)
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.pad = stride, pad
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = _Conv2d.apply(dy, w, ctx.stride, ctx.pad, tuple(x.shape[2:]))
        if ctx.needs_input_grad[1] and not weight_gradients_disabled:
            dw = _WGrad.apply(x, dy, tuple(w.shape[2:]), ctx.stride, ctx.pad).to(w.dtype)
        return dx, dw, None, None, None


class _WGrad(torch.autograd.Function):
    """dw[a, b, ky, kx] = sum_{n,p} g[n, a, p] * x[n, b, p*s + k - pad]  (f32 result)."""

    @staticmethod
    def forward(ctx, g, x, ksize, stride, pad):
        g, x = _nhwc(g), _nhwc(x)
        ctx.save_for_backward(g, x)
        ctx.stride, ctx.pad = stride, pad
        return _wgrad_raw(g, x, ksize[0], ksize[1], stride, pad)

    @staticmethod
    def backward(ctx, ddw):
        g, x = ctx.saved_tensors
        ddw = ddw.to(g.dtype)
        dg = dx = None
        if ctx.needs_input_grad[0]:
            dg = _Conv2d.apply(x, ddw, ctx.stride, ctx.pad, tuple(g.shape[2:]))
        if ctx.needs_input_grad[1]:
            dx = _ConvT2d.apply(g, ddw, ctx.stride, ctx.pad, tuple(x.shape[2:]))
        return dg, dx, None, None, None


def _depthwise_1d(x, w, groups, stride, py, px):
    """A depthwise 1-D correlation (one input and one output channel per group, a 1 x K or K x 1 kernel,
    stride 1, no padding): the ADA image filter (augment_mi.py _filter, groups = N * C, per-sample taps)."""
    return (groups == x.shape[1] == w.shape[0] and w.shape[1] == 1 and (w.shape[2] == 1 or w.shape[3] == 1)
            and stride == 1 and py == 0 and px == 0 and w.shape[2] * w.shape[3] <= 64)


def _depthwise_1d_conv(x, w):
    """y[:, g] = sum_t w[g, 0, t] * x[:, g, shifted by t] as K differentiable multiply-adds over the whole
    tensor (K launches) instead of one conv launch per group (N * C launches)."""
    kh, kw = w.shape[2], w.shape[3]
    k = kh * kw
    oh, ow = x.shape[2] - kh + 1, x.shape[3] - kw + 1
    taps = w.reshape(1, -1, k, 1, 1).to(x.dtype)
    y = None
    for t in range(k):
        xs = x[:, :, t:t + oh, :] if kh > 1 else x[:, :, :, t:t + ow]
        term = xs * taps[:, :, t]
        y = term if y is None else y + term
    return y


def conv2d(input, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
    """torch.nn.functional.conv2d semantics (correlation)."""
    _hip.require_device(input, weight)
    assert _pair(dilation) == (1, 1), 'dilation is not supported'
    sy, sx = _pair(stride)
    assert sy == sx, 'anisotropic stride is not supported'
    py, px = _pair(padding)
    if groups != 1 and _depthwise_1d(input, weight, groups, sy, py, px):
        y = _depthwise_1d_conv(input, weight)
    elif groups != 1:
        xs = input.chunk(groups, dim=1)
        ws = weight.chunk(groups, dim=0)
        y = torch.cat([conv2d(a, b_, None, stride, padding) for a, b_ in zip(xs, ws)], dim=1)
    else:
        n, c, h, w = input.shape
        o, i, kh, kw = weight.shape
        oh = (h + 2 * py - kh) // sy + 1
        ow = (w + 2 * px - kw) // sx + 1
        y = _Conv2d.apply(input, weight, sy, (py, px), (oh, ow))
    if bias is not None:
        y = y + bias.reshape(1, -1, 1, 1)
    return y


def conv_transpose2d(input, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1):
    """torch.nn.functional.conv_transpose2d semantics."""
    _hip.require_device(input, weight)
    assert _pair(dilation) == (1, 1), 'dilation is not supported'
    sy, sx = _pair(stride)
    assert sy == sx, 'anisotropic stride is not supported'
    py, px = _pair(padding)
    opy, opx = _pair(output_padding)
    if groups != 1:
        xs = input.chunk(groups, dim=1)
        ws = weight.chunk(groups, dim=0)
        y = torch.cat([conv_transpose2d(a, b_, None, stride, padding, output_padding) for a, b_ in zip(xs, ws)], dim=1)
    else:
        n, c, h, w = input.shape
        i, o, kh, kw = weight.shape
        oh = (h - 1) * sy - 2 * py + kh + opy
        ow = (w - 1) * sx - 2 * px + kw + opx
        y = _ConvT2d.apply(input, weight, sy, (py, px), (oh, ow))
    if bias is not None:
        y = y + bias.reshape(1, -1, 1, 1)
    return y
