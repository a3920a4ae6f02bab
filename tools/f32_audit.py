"""Per-call accuracy audit of the f32 convolutions (GPU): runs a phase-isolated fixture through the product with
conv_fused / _conv_raw / _wgrad_raw wrapped, recomputes every f32 call in float64 (torch, on the GPU) and lists
the calls whose relative error is above a threshold, with the calling line -- to find a conv form whose f32
arithmetic is short of f32 accuracy.

    python tools/f32_audit.py c2 [threshold]"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import config_parity as cp  # noqa: E402
from golden_util import load  # noqa: E402
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

ROWS = []
PHASE = {'name': None}


def _site():
    for fr in reversed(traceback.extract_stack()[:-3]):
        if 'conv2d_gradfix' not in fr.filename and 'f32_audit' not in fr.filename:
            return f'{os.path.basename(fr.filename)}:{fr.lineno}'
    return '?'


def _rel(a, b):
    return float((a.double() - b).norm() / max(float(b.norm()), 1e-300))


def _w_unpack(wp, transpose):
    w = wp.double()
    return w.permute(3, 0, 1, 2) if transpose else w.permute(0, 3, 1, 2)   # [I,O,kh,kw] / [O,I,kh,kw]


def _conv_ref(x, wp, oh, ow, stride, pad, transpose):
    w = _w_unpack(wp, transpose)
    if transpose:
        h, wd = x.shape[2:]
        op = (oh - ((h - 1) * stride - 2 * pad[0] + w.shape[2]), ow - ((wd - 1) * stride - 2 * pad[1] + w.shape[3]))
        return F.conv_transpose2d(x, w, stride=stride, padding=tuple(pad), output_padding=op)
    return F.conv2d(x, w, stride=stride, padding=tuple(pad))


def _record(kind, shape, err, extra=''):
    ROWS.append((err, kind, PHASE['name'], shape, _site(), extra))


_orig_fused, _orig_raw, _orig_wg = cg.conv_fused, cg._conv_raw, cg._wgrad_raw


def conv_fused(x, wp, cout, oh, ow, kh, kw, stride, pad, transpose=False, in_scale=None, out_scale=None, noise=None,
               noise_gain=1.0, bias=None, act=0, alpha=0.2, gain=1.0, clamp=-1.0, residual=None, aux_mode=0,
               dot_src=None, dot_out=None):
    res = _orig_fused(x, wp, cout, oh, ow, kh, kw, stride, pad, transpose, in_scale, out_scale, noise, noise_gain,
                      bias, act, alpha, gain, clamp, residual, aux_mode, dot_src, dot_out)
    if x.dtype != torch.float32:
        return res
    torch.cuda.synchronize()
    xd = x.double()
    if in_scale is not None:
        xd = xd * in_scale.double()[:, :, None, None]
    raw = _conv_ref(xd, wp, oh, ow, stride, pad, transpose)
    v = raw * (out_scale.double()[:, :, None, None] if out_scale is not None else 1.0)
    if noise is not None:
        nz = noise.double()
        v = v + nz.reshape(-1 if nz.numel() == v.shape[0] * oh * ow else 1, 1, oh, ow) * noise_gain
    if bias is not None:
        v = v + bias.double()[None, :, None, None]
    pre = v
    if act == 1:
        v = torch.where(v > 0, v, v * alpha)
    v = v * gain
    if clamp >= 0:
        v = v.clamp(-clamp, clamp)
    if residual is not None:
        v = v + residual.double()
    geom = (tuple(x.shape), cout, kh, stride, tuple(pad), 'T' if transpose else '')
    _record('fused.y', geom, _rel(res[0], v), f'act{act} aux{aux_mode} insc{in_scale is not None} '
            f'outsc{out_scale is not None}')
    if aux_mode == 1 and res[1] is not None:
        _record('fused.aux_raw', geom, min(_rel(res[1], raw), _rel(res[1], pre)))
    if dot_src is not None:
        ds = dot_src.double()
        cands = [(raw * ds).sum([2, 3]), (pre * ds).sum([2, 3]),
                 (raw * (out_scale.double()[:, :, None, None] if out_scale is not None else 1.0) * ds).sum([2, 3])]
        _record('fused.dot', geom, min(_rel(res[2], c) for c in cands))
    return res


def _conv_raw(x, wp, cout, oh, ow, kh, kw, stride, pad, transpose):
    y = _orig_raw(x, wp, cout, oh, ow, kh, kw, stride, pad, transpose)
    if x.dtype == torch.float32:
        torch.cuda.synchronize()
        _record('raw', (tuple(x.shape), cout, kh, stride, tuple(pad), 'T' if transpose else ''),
                _rel(y, _conv_ref(x.double(), wp, oh, ow, stride, pad, transpose)))
    return y


def _wgrad_raw(g, x, kh, kw, stride, pad, x_scale=None, g_scale=None, alpha=1.0, out=None):
    prev = out.clone() if out is not None else None
    dw = _orig_wg(g, x, kh, kw, stride, pad, x_scale, g_scale, alpha, out)
    if g.dtype == torch.float32:
        torch.cuda.synchronize()
        gd, xd = g.double(), x.double()
        if g_scale is not None:
            gd = gd * g_scale.double()[:, :, None, None]
        if x_scale is not None:
            xd = xd * x_scale.double()[:, :, None, None]
        # dw[a, b] = sum g[n, a, p] x[n, b, p*s + k - pad]: the weight gradient of conv2d(x, w) with output g
        ref = torch.nn.grad.conv2d_weight(xd, (g.shape[1], x.shape[1], kh, kw), gd, stride=stride, padding=tuple(pad))
        ref = ref * alpha
        got = dw.double() - (prev.view(g.shape[1], kh, kw, x.shape[1]).permute(0, 3, 1, 2).double()
                             if prev is not None else 0.0)
        _record('wgrad', (tuple(g.shape), tuple(x.shape), kh, stride, tuple(pad)), _rel(got, ref),
                f'gsc{g_scale is not None} xsc{x_scale is not None}')
    return dw


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else 'c2'
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 3e-6
    cg.conv_fused, cg._conv_raw, cg._wgrad_raw = conv_fused, _conv_raw, _wgrad_raw
    from training import loss as L
    orig_acc = L.StyleGAN2Loss.accumulate_gradients

    def acc(self, *a, **k):
        PHASE['name'] = k.get('phase', a[0] if a else None)
        try:
            return orig_acc(self, *a, **k)
        finally:
            PHASE['name'] = None
    L.StyleGAN2Loss.accumulate_gradients = acc
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}_iso.npz'))
    cp.run_product(cfg, inp, tape, torch.device('cuda', 0), aug_p=cfg['aug_p'], isolated=True)
    by = collections.defaultdict(list)
    for r in ROWS:
        by[(r[1], r[2])].append(r[0])
    print('calls per (kind, phase): max / median rel err')
    for k in sorted(by):
        v = sorted(by[k])
        print(f'  {k}: n {len(v)} max {v[-1]:.3g} median {v[len(v) // 2]:.3g}')
    print(f'calls above {thr:g}:')
    for r in sorted(ROWS, reverse=True):
        if r[0] > thr:
            print(f'  {r[0]:.3g} {r[1]:14s} {r[2]} {r[3]} {r[4]} {r[5]}')


if __name__ == '__main__':
    main()
