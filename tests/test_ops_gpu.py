"""Parity of the HIP ops (called through the C-ABI via the product wrappers) against the CPU oracle,
the reference's golden vectors, and torch-fp32 references for the convolution kernels.

Tolerances (relative L2 error):
  fp32 elementwise / FIR / grid_sample: 1e-5     fp32 MFMA convolutions: 1e-5
  fp16/bf16 (fp32 accumulate) vs the fp32 reference: 1e-2 (fp16), 2e-2 (bf16)
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from golden_util import load, lit, rel_err
from rngtape import Tape
from oracle import sg2_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


def T(a, dev=DEV, rg=False):
    return torch.from_numpy(np.array(a, dtype=np.float32)).to(dev).requires_grad_(rg)


# ------------------------------------------------------------------ bias_act
BA = load('bias_act.npz')


@pytest.mark.parametrize('name', [str(n) for n in BA['names']])
def test_bias_act_golden(name):
    from torch_utils.ops import bias_act
    z = BA
    act, g, c = name.split('_g')[0], name.split('_g')[1].split('_c')[0], name.split('_c')[1]
    gain = None if g == 'None' else float(g)
    clamp = None if c == 'None' else float(c)
    for fmt in [torch.contiguous_format, torch.channels_last]:
        x = T(z['x']).contiguous(memory_format=fmt).requires_grad_(True)
        b = T(z['b'], rg=True)
        y = bias_act.bias_act(x, b, act=act, gain=gain, clamp=clamp)
        assert rel_err(y, z[f'{name}_y']) < 1e-5
        gx, gb = torch.autograd.grad((y * T(z['dy'])).sum(), [x, b], create_graph=True)
        assert rel_err(gx, z[f'{name}_dx']) < 1e-5
        assert rel_err(gb, z[f'{name}_db']) < 1e-5
        if f'{name}_ddx' in z.files:
            hx, = torch.autograd.grad((gx * T(z['v'])).sum(), [x])
            assert rel_err(hx, z[f'{name}_ddx']) < 1e-4


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
def test_bias_act_lowp(dtype):
    from torch_utils.ops import bias_act
    x = torch.randn(4, 64, 9, 11, device=DEV).contiguous(memory_format=torch.channels_last)
    b = torch.randn(64, device=DEV)
    y = bias_act.bias_act(x.to(dtype), b.to(dtype), act='lrelu', gain=np.sqrt(2), clamp=256)
    r = O.bias_act(x.cpu(), b.cpu(), act='lrelu', gain=np.sqrt(2), clamp=256)
    assert rel_err(y.float(), r) < (1e-2 if dtype == torch.float16 else 2e-2)


def test_bias_act_odd_sizes():
    from torch_utils.ops import bias_act
    for shape in [(3, 5), (1, 7, 3, 3), (2, 3, 1, 13)]:
        x = torch.randn(*shape, device=DEV)
        b = torch.randn(shape[1], device=DEV)
        y = bias_act.bias_act(x, b, act='swish', clamp=0.5)
        assert rel_err(y, O.bias_act(x.cpu(), b.cpu(), act='swish', clamp=0.5)) < 1e-5


def test_rejects_cpu():
    from torch_utils.ops import bias_act, upfirdn2d
    with pytest.raises(RuntimeError):
        bias_act.bias_act(torch.zeros(2, 3))
    with pytest.raises(RuntimeError):
        upfirdn2d.upfirdn2d(torch.zeros(1, 1, 4, 4), None)


# ------------------------------------------------------------------ upfirdn2d
UPF = load('upfirdn2d.npz')


@pytest.mark.parametrize('name', [str(n) for n in UPF['names']])
@pytest.mark.parametrize('fmt', ['nchw', 'nhwc'])
def test_upfirdn2d_golden(name, fmt):
    from torch_utils.ops import upfirdn2d
    z = UPF
    kw = lit(z, f'{name}_kw')
    f = z[f'{name}_f']
    f = None if f.size == 0 else torch.from_numpy(f).to(DEV)
    x = T(z[f'{name}_x'])
    if fmt == 'nhwc':
        x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = upfirdn2d.upfirdn2d(x, f, **kw)
    assert rel_err(y, z[f'{name}_y']) < 1e-5
    dx, = torch.autograd.grad((y * T(z[f'{name}_dy'])).sum(), [x])
    assert rel_err(dx, z[f'{name}_dx']) < 1e-5


@pytest.mark.parametrize('kw', [dict(up=2, padding=[6, 5, 6, 5]), dict(up=2, padding=[5, 4, 7, 3]),
                                dict(down=2, padding=[-3, -2, -3, -4]), dict(down=2, padding=[2, 3, 1, 5]),
                                dict(up=2, padding=[1, 2, 0, 3], flip_filter=True), dict(padding=[5, 6, 5, 6])])
def test_upfirdn2d_separable_passes(kw):
    """The 1-D passes of a separable (1-D) filter on f32 NCHW images (upfirdn_1d, and upfirdn_1d_vrun for the
    vertical up-2 / down-2 passes of the 12-tap ADA filter: runs of 4 output rows, both pad parities), forward
    and input gradient vs the oracle; several planes, ragged sizes (a partial last run and column tile)."""
    from torch_utils.ops import upfirdn2d
    torch.manual_seed(11)
    f = torch.randn(12, dtype=torch.float64)
    x = torch.randn(3, 2, 37, 301, dtype=torch.float64)
    xd = x.float().to(DEV).requires_grad_(True)
    y = upfirdn2d.upfirdn2d(xd, f.float().to(DEV), **kw)
    r = O.upfirdn2d(x, f, **kw)
    assert y.shape == r.shape
    assert rel_err(y, r) < 1e-5
    dy = torch.randn(r.shape, dtype=torch.float64)
    dx, = torch.autograd.grad((y * dy.float().to(DEV)).sum(), [xd])
    xr = x.clone().requires_grad_(True)
    ref, = torch.autograd.grad((O.upfirdn2d(xr, f, **kw) * dy).sum(), [xr])
    assert rel_err(dx, ref) < 1e-5


@pytest.mark.parametrize('dtype', [torch.float32, torch.float16, torch.bfloat16])
def test_upfirdn2d_vec_path(dtype):
    """Channel-vectorised NHWC kernel on network-shaped tensors, vs the oracle in fp32."""
    from torch_utils.ops import upfirdn2d
    f = upfirdn2d.setup_filter([1, 3, 3, 1])
    x = torch.randn(2, 64, 17, 17)
    cases = [dict(padding=[1, 1, 1, 1], gain=4), dict(padding=[2, 2, 2, 2]), dict(down=2, padding=[1, 1, 1, 1]),
             dict(up=2, padding=[2, 1, 2, 1], gain=4)]
    tol = {torch.float32: 1e-5, torch.float16: 2e-3, torch.bfloat16: 1e-2}[dtype]
    for kw in cases:
        xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
        y = upfirdn2d.upfirdn2d(xd, f.to(DEV), **kw)
        r = O.upfirdn2d(x.to(dtype).float(), f, **kw)
        assert rel_err(y.float(), r) < tol, kw


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
def test_upfirdn2d_f4s_c32(dtype, monkeypatch):
    """The 4x4 FIR strip kernel's C = 32 form (16-bit: a 64-byte pixel, 64-column tiles of 4 channel vectors; C5's
    1024^2 layers) vs the oracle, plain and with the fused layer epilogue, and bitwise against the 8-vector-group
    form (SG2_FIR_C32=0: the same taps in the same order)."""
    from torch_utils.ops import upfirdn2d
    torch.manual_seed(9)
    tol = {torch.float16: 2e-3, torch.bfloat16: 1e-2}[dtype]
    f = upfirdn2d.setup_filter([1, 3, 3, 1])
    for (n, h, w, pad) in [(2, 24, 128, [2, 1, 2, 1]), (1, 40, 256, [2, 2, 2, 2]), (3, 9, 227, [1, 2, 2, 1])]:
        x = torch.randn(n, 32, h, w).to(dtype).float()
        xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
        monkeypatch.delenv('SG2_FIR_C32', raising=False)
        y = upfirdn2d.upfirdn2d(xd, f.to(DEV), padding=pad, gain=4)
        r = O.upfirdn2d(x, f, padding=pad, gain=4)
        assert y.shape == r.shape
        assert rel_err(y.float(), r) < tol, (n, h, w, pad)
        f2 = f.to(DEV)                                 # (setup_filter makes the 4-tap filter 2-D)
        s = (torch.rand(n, 32) + 0.5).to(DEV)
        b = (torch.randn(32) * 0.1).to(DEV)
        ye, _ = upfirdn2d.fir_fused(xd, f2, pad, gain=4.0, out_scale=s, bias=b, act=1, alpha=0.2,
                                    act_gain=2 ** 0.5, clamp=256.0)
        monkeypatch.setenv('SG2_FIR_C32', '0')
        assert torch.equal(y, upfirdn2d.upfirdn2d(xd, f.to(DEV), padding=pad, gain=4)), (n, h, w, pad)
        ye2, _ = upfirdn2d.fir_fused(xd, f2, pad, gain=4.0, out_scale=s, bias=b, act=1, alpha=0.2,
                                     act_gain=2 ** 0.5, clamp=256.0)
        assert torch.equal(ye, ye2), (n, h, w, pad)


@pytest.mark.parametrize('dtype', [torch.float32, torch.float16, torch.bfloat16])
def test_upfirdn2d_up2_blocks(dtype, monkeypatch):
    """2x up-FIR on channels-last feature maps (upfirdn_nhwc_up2, a 2 x 2 output cell per lane; the adjoint of
    the D skip's FIR-down-2): even / odd / asymmetric / zero padding, odd output sizes, flipped and asymmetric
    filters, vs the oracle, and bitwise against the per-output kernel it replaced (upfirdn_nhwc_vec,
    SG2_UPF_UP2_OFF=1; same taps in the same order).  (Round 2's LDS-staged 2 x 2-block kernel measured 1.8x
    slower, profiles/r02_v9_fir_up2_ab.log; this register form is 1.5-1.7x faster, profiles/r04_v4_upf_up2_ab.log.)"""
    from torch_utils.ops import upfirdn2d
    torch.manual_seed(5)
    tol = {torch.float32: 1e-5, torch.float16: 2e-3, torch.bfloat16: 1e-2}[dtype]
    for fk in ([1, 3, 3, 1], [1, 2, 5, 3]):
        f = upfirdn2d.setup_filter(fk)
        for (n, c, h, w) in [(2, 64, 17, 17), (1, 32, 16, 9), (3, 128, 8, 8)]:
            x = torch.randn(n, c, h, w).to(dtype).float()
            xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
            for pad in ([2, 1, 2, 1], [1, 2, 1, 2], [2, 2, 2, 2], [1, 1, 1, 1], [0, 0, 0, 0], [3, 0, 1, 2]):
                for flip in (False, True):
                    y = upfirdn2d.upfirdn2d(xd, f.to(DEV), up=2, padding=pad, flip_filter=flip, gain=4)
                    r = O.upfirdn2d(x, f, up=2, padding=pad, flip_filter=flip, gain=4)
                    assert y.shape == r.shape
                    assert rel_err(y.float(), r) < tol, (fk, n, c, h, w, pad, flip)
                    monkeypatch.setenv('SG2_UPF_UP2_OFF', '1')
                    y2 = upfirdn2d.upfirdn2d(xd, f.to(DEV), up=2, padding=pad, flip_filter=flip, gain=4)
                    monkeypatch.delenv('SG2_UPF_UP2_OFF')
                    assert torch.equal(y, y2), (fk, n, c, h, w, pad, flip)


@pytest.mark.parametrize('dtype', [torch.float32, torch.float16, torch.bfloat16])
def test_fir_strip_ragged(dtype):
    """Column-strip FIR kernel (upfirdn_nhwc_f4s): image sizes that are not tile multiples (the last
    tile row/column is shifted back inside the image), partial channel groups (C = 72), plain and
    with the full layer epilogue (out_scale, noise, bias, lrelu, gain, clamp, aux), vs the oracle."""
    from torch_utils.ops import upfirdn2d
    torch.manual_seed(3)
    f = upfirdn2d.setup_filter([1, 3, 3, 1])
    tol = {torch.float32: 1e-5, torch.float16: 2e-3, torch.bfloat16: 1e-2}[dtype]
    for (n, c, h, w, pad) in [(2, 64, 45, 250, 1), (1, 128, 33, 40, 2), (2, 72, 20, 33, 1), (1, 64, 257, 257, 1)]:
        x = torch.randn(n, c, h, w).to(dtype).float()
        xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
        ref = O.upfirdn2d(x, f, padding=pad, gain=4)
        y = upfirdn2d.upfirdn2d(xd, f.to(DEV), padding=pad, gain=4)
        assert rel_err(y.float(), ref) < tol, (n, c, h, w, pad)
        oh, ow = ref.shape[2:]
        os_ = torch.rand(n, c) + 0.5
        noise = torch.randn(n, 1, oh, ow).to(dtype).float()
        bias = torch.randn(c).to(dtype).float()
        for aux_mode in (1, 2):
            yd, aux = upfirdn2d.fir_fused(xd, f.to(DEV), pad, gain=4, out_scale=os_.to(DEV), noise=noise.to(DEV, dtype),
                                          noise_gain=0.3, bias=bias.to(DEV), act=1, alpha=0.2, act_gain=1.4,
                                          clamp=2.5, aux_mode=aux_mode)
            z = ref * os_[:, :, None, None] + noise * 0.3 + bias[None, :, None, None]
            z = (torch.where(z > 0, z, z * 0.2) * 1.4).clamp(-2.5, 2.5)
            assert rel_err(yd.float(), z) < tol, (n, c, h, w, pad, aux_mode)
            assert rel_err(aux.float(), ref if aux_mode == 1 else z) < tol, (n, c, h, w, pad, aux_mode)


# ------------------------------------------------------------------ convolutions (torch fp32 reference)
CONV_CASES = [
    # N, Cin, H, W, Cout, k, stride, pad
    (2, 64, 16, 16, 64, 3, 1, 1),
    (2, 32, 9, 9, 48, 3, 2, 0),
    (3, 16, 8, 8, 24, 1, 1, 0),
    (2, 1, 8, 8, 16, 1, 1, 0),
    (2, 16, 8, 8, 1, 1, 1, 0),
    (2, 64, 6, 6, 3, 1, 1, 0),
    (2, 3, 10, 10, 8, 3, 1, 1),
    (2, 13, 7, 7, 130, 3, 1, 1),
    (2, 513, 4, 4, 64, 3, 1, 1),
    (1, 128, 4, 4, 256, 3, 1, 1),
    (32, 512, 4, 4, 512, 3, 1, 1),
]


def _ref_conv(x, w, stride, pad, transpose=False, out_hw=None):
    x, w = x.double().cpu(), w.double().cpu()
    if transpose:
        y = F.conv_transpose2d(x, w, stride=stride, padding=pad)
        if out_hw is not None and tuple(y.shape[2:]) != tuple(out_hw):
            op = (out_hw[0] - y.shape[2], out_hw[1] - y.shape[3])
            y = F.conv_transpose2d(x, w, stride=stride, padding=pad, output_padding=op)
        return y
    return F.conv2d(x, w, stride=stride, padding=pad)


@pytest.mark.parametrize('case', CONV_CASES)
@pytest.mark.parametrize('dtype', [torch.float32, torch.float16, torch.bfloat16])
def test_conv2d_fwd_bwd(case, dtype):
    from torch_utils.ops import conv2d_gradfix as cg
    N, Cin, H, W, Cout, k, s, p = case
    torch.manual_seed(0)
    x = torch.randn(N, Cin, H, W)
    w = torch.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)
    tol = {torch.float32: 1e-5, torch.float16: 4e-3, torch.bfloat16: 2e-2}[dtype]
    xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wd = w.to(DEV, dtype).requires_grad_(True)
    y = cg.conv2d(xd, wd, stride=s, padding=p)
    xr, wr = x.to(dtype).double(), w.to(dtype).double()
    yr = _ref_conv(xr, wr, s, p)
    assert y.shape == yr.shape
    assert rel_err(y.float(), yr) < tol
    dy = torch.randn(y.shape)
    gx, gw = torch.autograd.grad(y, [xd, wd], dy.to(DEV, dtype))
    xr.requires_grad_(True)
    wr.requires_grad_(True)
    gxr, gwr = torch.autograd.grad(F.conv2d(xr, wr, stride=s, padding=p), [xr, wr], dy.to(dtype).double())
    assert rel_err(gx.float(), gxr) < tol
    assert rel_err(gw.float(), gwr) < tol * 2


@pytest.mark.parametrize('case', [(2, 64, 8, 8, 64, 3, 2, 0), (2, 16, 5, 5, 8, 3, 2, 1), (2, 32, 4, 4, 32, 1, 1, 0),
                                  (4, 512, 4, 4, 512, 3, 2, 0), (2, 24, 6, 6, 40, 3, 1, 1)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.float16])
def test_conv_transpose2d(case, dtype):
    from torch_utils.ops import conv2d_gradfix as cg
    N, Cin, H, W, Cout, k, s, p = case
    torch.manual_seed(1)
    x = torch.randn(N, Cin, H, W)
    w = torch.randn(Cin, Cout, k, k) / np.sqrt(Cin * k * k)
    tol = {torch.float32: 1e-5, torch.float16: 4e-3}[dtype]
    xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wd = w.to(DEV, dtype).requires_grad_(True)
    y = cg.conv_transpose2d(xd, wd, stride=s, padding=p)
    xr, wr = x.to(dtype).double().requires_grad_(True), w.to(dtype).double().requires_grad_(True)
    yr = F.conv_transpose2d(xr, wr, stride=s, padding=p)
    assert y.shape == yr.shape
    assert rel_err(y.float(), yr.detach()) < tol
    dy = torch.randn(y.shape)
    gx, gw = torch.autograd.grad(y, [xd, wd], dy.to(DEV, dtype))
    gxr, gwr = torch.autograd.grad(yr, [xr, wr], dy.to(dtype).double())
    assert rel_err(gx.float(), gxr) < tol
    assert rel_err(gw.float(), gwr) < tol * 2


def test_conv_double_backward():
    """Second order through conv (the PL / R1 path): d/dw <dL/dx, v> vs torch fp64 on CPU."""
    from torch_utils.ops import conv2d_gradfix as cg
    torch.manual_seed(2)
    x = torch.randn(2, 16, 8, 8)
    w = torch.randn(24, 16, 3, 3) / 12
    v = torch.randn(2, 16, 8, 8)
    res = []
    for dev, dt in [(DEV, torch.float32), (torch.device('cpu'), torch.float64)]:
        xd = x.to(dev, dt).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        wd = w.to(dev, dt).requires_grad_(True)
        fn = cg.conv2d if dev.type == 'cuda' else F.conv2d
        y = fn(xd, wd, stride=1, padding=1)
        l1 = (y.square()).sum()
        gx, = torch.autograd.grad(l1, [xd], create_graph=True)
        gw2, gx2 = torch.autograd.grad((gx * v.to(dev, dt)).sum(), [wd, xd])
        res.append((gw2.double().cpu(), gx2.double().cpu()))
    assert rel_err(res[0][0], res[1][0]) < 1e-5
    assert rel_err(res[0][1], res[1][1]) < 1e-5


# ------------------------------------------------------------------ grid_sample
def test_grid_sample():
    from torch_utils.ops import grid_sample_gradfix as gs
    torch.manual_seed(3)
    x = torch.randn(2, 3, 20, 24)
    theta = torch.tensor([[[1.05, 0.1, 0.03], [-0.08, 0.95, -0.02]], [[0.9, -0.2, 0.1], [0.15, 1.1, 0.05]]])
    grid = F.affine_grid(theta, [2, 3, 30, 26], align_corners=False)
    xd = x.to(DEV).requires_grad_(True)
    y = gs.grid_sample(xd, grid.to(DEV))
    yr = F.grid_sample(x.double(), grid.double(), mode='bilinear', padding_mode='zeros', align_corners=False)
    assert rel_err(y, yr) < 1e-5
    dy = torch.randn(y.shape)
    dyd = dy.to(DEV).requires_grad_(True)
    gx, = torch.autograd.grad(y, [xd], dyd, create_graph=True)
    xr = x.double().requires_grad_(True)
    gxr, = torch.autograd.grad(F.grid_sample(xr, grid.double(), align_corners=False), [xr], dy.double())
    assert rel_err(gx, gxr) < 1e-5
    # backward-of-backward w.r.t. the incoming gradient = forward sampling of v
    v = torch.randn(gx.shape)
    ggo, = torch.autograd.grad((gx * v.to(DEV)).sum(), [dyd])
    assert rel_err(ggo, F.grid_sample(v.double(), grid.double(), align_corners=False)) < 1e-5



def test_affine_grid_sample():
    """Grid built inside the kernel (sg2_affine_grid_sample_*) vs affine_grid + grid_sample in fp64:
    forward, input gradient, backward-of-backward; also with a static buffer + dyn_hw."""
    from torch_utils.ops import grid_sample_gradfix as gs
    torch.manual_seed(4)
    x = torch.randn(2, 1, 40, 36)
    theta = torch.tensor([[[1.05, 0.1, 0.03], [-0.08, 0.95, -0.02]], [[0.9, -0.2, 0.1], [0.15, 1.1, 0.05]]])
    size = [2, 1, 50, 46]
    grid = F.affine_grid(theta.double(), size, align_corners=False)
    xd = x.to(DEV).requires_grad_(True)
    y = gs.affine_grid_sample(xd, theta.to(DEV), size)
    assert rel_err(y, F.grid_sample(x.double(), grid, align_corners=False)) < 1e-5
    dy = torch.randn(y.shape)
    dyd = dy.to(DEV).requires_grad_(True)
    gx, = torch.autograd.grad(y, [xd], dyd, create_graph=True)
    xr = x.double().requires_grad_(True)
    gxr, = torch.autograd.grad(F.grid_sample(xr, grid, align_corners=False), [xr], dy.double())
    assert rel_err(gx, gxr) < 1e-5
    v = torch.randn(gx.shape)
    ggo, = torch.autograd.grad((gx * v.to(DEV)).sum(), [dyd])
    assert rel_err(ggo, F.grid_sample(v.double(), grid, align_corners=False)) < 1e-5
    # logical 30 x 28 image at the origin of the 40 x 36 buffer
    dyn = torch.tensor([30, 28], dtype=torch.int32, device=DEV)
    y2 = gs.affine_grid_sample(xd, theta.to(DEV), size, dyn_hw=dyn)
    assert rel_err(y2, F.grid_sample(x[:, :, :30, :28].double(), grid, align_corners=False)) < 1e-5

# ------------------------------------------------------------------ modulated conv + conv layers (golden)
CV = load('conv.npz')


@pytest.mark.parametrize('name', [str(n) for n in CV['names'] if str(n).startswith('modconv')])
def test_modconv_golden(name):
    from training import networks_stylegan2 as net
    from torch_utils.ops import upfirdn2d
    z = CV
    up = int(name.split('_up')[1][0])
    demod = bool(int(name.split('_d')[1][0]))
    fused = bool(int(name.split('_f')[1][0]))
    x, w, s, nz = (T(z[f'{name}_{k}'], rg=True) for k in ['x', 'w', 's', 'noise'])
    y = net.modulated_conv2d(x, w, s, noise=nz, up=up, padding=1,
                             resample_filter=upfirdn2d.setup_filter([1, 3, 3, 1]).to(DEV), demodulate=demod,
                             flip_weight=(up == 1), fused_modconv=fused)
    assert rel_err(y, z[f'{name}_y']) < 1e-5
    grads = torch.autograd.grad((y * T(z[f'{name}_dy'])).sum(), [x, w, s, nz])
    for k, g in zip(['dx', 'dw', 'ds', 'dnoise'], grads):
        assert rel_err(g, z[f'{name}_{k}']) < 1e-5, k


@pytest.mark.parametrize('name', [str(n) for n in CV['names'] if not str(n).startswith('modconv')])
def test_conv_layer_golden(name):
    from training import networks_stylegan2 as net
    z = CV
    layer = net.Conv2dLayer(**lit(z, f'{name}_kw')).to(DEV)
    with torch.no_grad():
        layer.weight.copy_(T(z[f'{name}_w']))
        if layer.bias is not None:
            layer.bias.copy_(T(z[f'{name}_b']))
    x = T(z[f'{name}_x'], rg=True)
    y = layer(x, gain=float(z[f'{name}_gain']))
    assert rel_err(y, z[f'{name}_y']) < 1e-5
    params = [x, layer.weight] + ([layer.bias] if layer.bias is not None else [])
    grads = torch.autograd.grad((y * T(z[f'{name}_dy'])).sum(), params)
    assert rel_err(grads[0], z[f'{name}_dx']) < 1e-5
    assert rel_err(grads[1], z[f'{name}_dw']) < 1e-5
    if layer.bias is not None:
        assert rel_err(grads[2], z[f'{name}_db']) < 1e-5


# ------------------------------------------------------------------ augment pipe (golden)
AU = load('augment.npz')


@pytest.mark.parametrize('name', [str(n) for n in AU['names']])
def test_augment_golden(name):
    from training import augment_mi
    z = AU
    cfg = lit(z, f'{name.split("_")[0]}_cfg')
    pipe = augment_mi.AugmentPipe(run_dir=None, batch_size=2, **cfg).to(DEV)
    x = T(z[f'{name}_x'], rg=True)
    if name.endswith('_rand'):
        pipe.p.fill_(float(z[f'{name}_p']))
        tape = Tape.from_npz(z, prefix=f'{name}_tape')
        with tape.replay():
            y = pipe(x, False)
        assert tape.pos == len(tape.entries)
    elif any(k.startswith(f'{name}_tape') for k in z.files):    # the noise branch: pixel noise drawn at any percentile
        tape = Tape.from_npz(z, prefix=f'{name}_tape')
        with tape.replay():
            y = pipe(x, False, debug_percentile=float(name.split('_p')[1]))
        assert tape.pos == len(tape.entries)
    else:
        y = pipe(x, False, debug_percentile=float(name.split('_p')[1]))
    assert rel_err(y, z[f'{name}_y']) < 2e-5
    dx, = torch.autograd.grad((y * T(z[f'{name}_dy'])).sum(), [x])
    assert rel_err(dx, z[f'{name}_dx']) < 2e-5


@pytest.mark.parametrize('p,n', [(0.0, 4), (0.2, 64), (1.0, 300)])
def test_augment_geometric_fused_matches_torch_algebra(p, n, monkeypatch):
    """sg2_aug_geom (one launch for the transform algebra) against the per-op torch algebra it replaces, on the
    same draws: images and input gradients to 1e-5, every op of the pipe enabled (incl. rotate90), the batch
    beyond one workgroup's 256 threads (n = 300)."""
    from training import augment_mi
    cfg = dict(xflip=1, rotate90=1, xint=1, scale=1, rotate=1, aniso=1, xfrac=1, xint_max=0.05, rotate_max=3 / 360,
               xfrac_std=0.05, scale_std=0.05, aniso_std=0.05)
    pipe = augment_mi.AugmentPipe(run_dir=None, batch_size=n, **cfg).to(DEV)
    pipe.p.fill_(p)
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(n, 1, 32, 32, generator=g) * 2 - 1).to(DEV).requires_grad_(True)
    dy = torch.randn(n, 1, 32, 32, generator=g).to(DEV)
    out = []
    for fused in (True, False):
        monkeypatch.setattr(augment_mi, 'fused_geometric', fused)
        torch.manual_seed(123)
        y = pipe(x, False)
        dx, = torch.autograd.grad((y * dy).sum(), [x])
        out.append((y.detach(), dx))
    assert rel_err(out[0][0], out[1][0].double().cpu()) < 1e-5
    assert rel_err(out[0][1], out[1][1].double().cpu()) < 1e-5


# ------------------------------------------------------------------ LDS-halo 3x3 conv with fused epilogue
@pytest.mark.parametrize('shape', [(2, 64, 32, 32, 64), (2, 64, 20, 37, 96), (1, 512, 32, 32, 512), (2, 128, 16, 16, 128),
                                   (2, 40, 16, 24, 8),
                                   (4, 64, 256, 256, 64), (9, 64, 128, 256, 64)])   # persistent c64 kernel
@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
def test_conv3x3_fused(shape, dtype):
    from torch_utils.ops import conv2d_gradfix as cg
    N, Cin, H, W, Cout = shape
    torch.manual_seed(5)
    x = torch.randn(N, Cin, H, W)
    w = torch.randn(Cout, Cin, 3, 3) / np.sqrt(Cin * 9)
    s = torch.rand(N, Cin) + 0.5
    d = torch.rand(N, Cout) + 0.5
    noise = torch.randn(N, 1, H, W)
    b = torch.randn(Cout) * 0.1
    xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv(w.to(DEV, dtype))
    y, raw = cg.conv3x3_fused(xd, wp, Cout, in_scale=s.to(DEV), out_scale=d.to(DEV),
                              noise=noise.to(DEV, dtype).reshape(N, H, W).contiguous(), noise_gain=0.3,
                              bias=b.to(DEV), act=1, alpha=0.2, gain=np.sqrt(2), clamp=1.5, want_raw=True)
    xs = (x.to(dtype).float() * s[:, :, None, None]).to(dtype).double()
    c = F.conv2d(xs, w.to(dtype).double(), padding=1)
    z = c * d[:, :, None, None] + noise.to(dtype).double() * 0.3 + b[None, :, None, None]
    yr = (F.leaky_relu(z, 0.2) * np.sqrt(2)).clamp(-1.5, 1.5)
    tol = 5e-3 if dtype == torch.float16 else 2e-2
    assert rel_err(raw.float(), c) < tol
    assert rel_err(y.float(), yr) < tol


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(2, 64, 20, 37, 128), (1, 256, 33, 40, 192), (3, 128, 16, 16, 64),
                                   (2, 512, 32, 32, 512)])
@pytest.mark.parametrize('direct', ['1', '0'])
def test_conv3x3_halo_direct(dtype, shape, direct, monkeypatch):
    """The halo kernel's direct epilogue (conv3x3.hip DIR: swapped MFMA operands, p_chan weight rows, 16-byte
    stores from registers; direct '0': the LDS-transposed epilogue) against float64: the modulated layer with the
    full epilogue and its raw output, and the dgrad form (out_scale + dot) with float atomics and in
    deterministic mode.  Ragged tiles (20 x 37, 33 x 40), TW = 16 (16 x 16), 1..8 channel tiles."""
    import sg2hip
    from torch_utils.ops import conv2d_gradfix as cg
    monkeypatch.setenv('SG2_HALO_DIRECT', direct)
    monkeypatch.setenv('SG2_C64_RING', '0')
    N, Cin, H, W, Cout = shape
    torch.manual_seed(13)
    x = torch.randn(N, Cin, H, W)
    w = torch.randn(Cout, Cin, 3, 3) / np.sqrt(Cin * 9)
    s = torch.rand(N, Cin) + 0.5
    d = torch.rand(N, Cout) + 0.5
    noise = torch.randn(N, 1, H, W)
    b = torch.randn(Cout) * 0.1
    xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv(w.to(DEV, dtype))
    y, raw = cg.conv3x3_fused(xd, wp, Cout, in_scale=s.to(DEV), out_scale=d.to(DEV),
                              noise=noise.to(DEV, dtype).reshape(N, H, W).contiguous(), noise_gain=0.3,
                              bias=b.to(DEV), act=1, alpha=0.2, gain=np.sqrt(2), clamp=1.5, want_raw=True)
    xs = (x.to(dtype).float() * s[:, :, None, None]).to(dtype).double()
    c = F.conv2d(xs, w.to(dtype).double(), padding=1)
    z = c * d[:, :, None, None] + noise.to(dtype).double() * 0.3 + b[None, :, None, None]
    yr = (F.leaky_relu(z, 0.2) * np.sqrt(2)).clamp(-1.5, 1.5)
    tol = 5e-3 if dtype == torch.float16 else 2e-2
    assert rel_err(raw.float(), c) < tol and rel_err(y.float(), yr) < tol
    for n in range(N):
        assert rel_err(y[n].float(), yr[n]) < 2 * tol, n
    src = torch.randn(N, Cout, H, W).to(dtype)
    c0 = F.conv2d(x.to(dtype).double(), w.to(dtype).double(), padding=1)
    for det in (False, True):
        with sg2hip.deterministic(det, device=DEV):
            y, _, dot = cg.conv3x3_fused(xd, wp, Cout, out_scale=d.to(DEV),
                                         dot_src=src.to(DEV).contiguous(memory_format=torch.channels_last))
        assert rel_err(y.float(), c0 * d[:, :, None, None]) < tol
        assert rel_err(dot, (c0.to(dtype).double() * src.double()).sum([2, 3])) < tol


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
def test_fused_synthesis_layer_matches_composed(dtype):
    """SynthesisLayer through the one-kernel path (sg2_conv3x3 + ModConvLayer backward) vs the composed
    path (x*s, conv, fma, bias_act kernels): outputs, first-order grads and the PL-style second-order
    grads w.r.t. the parameters."""
    from training import networks_stylegan2 as net
    from torch_utils.ops import modconv
    torch.manual_seed(9)
    layer = net.SynthesisLayer(32, 48, w_dim=16, resolution=16, conv_clamp=256).to(DEV)
    with torch.no_grad():
        layer.noise_strength.fill_(0.3)
        layer.bias.copy_(torch.randn(48) * 0.2)
    x0 = torch.randn(4, 32, 16, 16, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    w0 = torch.randn(4, 16, device=DEV)
    noise = torch.randn(4, 1, 16, 16, device=DEV)
    pl = torch.randn(4, 48, 16, 16, device=DEV)
    res = []
    for fused in [True, False]:
        modconv.enabled = fused
        x = x0.clone().requires_grad_(True)
        wv = w0.clone().requires_grad_(True)
        orig = torch.randn
        torch.randn = lambda *a, **k: noise.clone()
        try:
            y = layer(x, wv)
        finally:
            torch.randn = orig
        params = [layer.weight, layer.bias, layer.noise_strength, layer.affine.weight, layer.affine.bias]
        for p_ in params:
            p_.requires_grad_(True)
        g_w, = torch.autograd.grad((y.float() * pl).sum(), [wv], create_graph=True)
        gx, = torch.autograd.grad((y.float() * pl).sum(), [x], retain_graph=True)
        g2 = torch.autograd.grad(g_w.square().sum(), params, allow_unused=True)
        res.append((y.float(), gx.float(), g_w.float(), [g if g is None else g.float() for g in g2]))
    modconv.enabled = True
    tol = 2e-2 if dtype == torch.float16 else 5e-2
    (y1, gx1, gw1, g21), (y2, gx2, gw2, g22) = res
    assert rel_err(y1, y2) < tol
    assert rel_err(gx1, gx2) < tol
    assert rel_err(gw1, gw2) < tol
    for a_, b_ in zip(g21, g22):
        if b_ is None:
            continue
        assert a_ is not None
        assert rel_err(a_, b_) < 4 * tol


@pytest.mark.parametrize('dtype,res', [(torch.float16, 16), (torch.bfloat16, 16), (torch.float32, 16),
                                       (torch.float16, 4), (torch.float32, 8)])
def test_fused_synthesis_layer_pl_pass(dtype, res, monkeypatch):
    """The path-length pass as loss.py runs it: the create_graph gradient w.r.t. ws under
    conv2d_gradfix.no_weight_gradients() (where the dgrad goes through _ScaledConvT, the demodulation scale
    on the operand staging), then the penalty's backward with weight gradients enabled (_ScaledConvT's
    backward: conv(G, W) * d with the dd dot epilogue, and the d-scaled wgrad).  Fused path vs the composed
    one (x*s, conv, fma, bias_act kernels) and against the fused layer's composed VJP (modconv.fused_vjp off);
    16-bit at 16^2 runs the halo kernels, f32 and 4^2 the generic."""
    from training import networks_stylegan2 as net
    from torch_utils.ops import conv2d_gradfix, modconv
    torch.manual_seed(13)
    layer = net.SynthesisLayer(32, 48, w_dim=16, resolution=res, conv_clamp=256).to(DEV)
    with torch.no_grad():
        layer.noise_strength.fill_(0.3)
        layer.bias.copy_(torch.randn(48) * 0.2)
    x0 = torch.randn(4, 32, res, res, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    w0 = torch.randn(4, 16, device=DEV)
    noise = torch.randn(4, 1, res, res, device=DEV)
    pl = torch.randn(4, 48, res, res, device=DEV)
    params = [layer.weight, layer.bias, layer.noise_strength, layer.affine.weight, layer.affine.bias]
    out = []
    for fused, vjp in [(True, True), (False, False), (True, False)]:
        monkeypatch.setattr(modconv, 'enabled', fused)
        monkeypatch.setattr(modconv, 'fused_vjp', vjp)
        x = x0.clone().requires_grad_(True)
        wv = w0.clone().requires_grad_(True)
        orig = torch.randn
        torch.randn = lambda *a, **k: noise.clone()
        try:
            y = layer(x, wv)
        finally:
            torch.randn = orig
        with conv2d_gradfix.no_weight_gradients():
            g_w, = torch.autograd.grad((y.float() * pl).sum(), [wv], create_graph=True)
        g2 = torch.autograd.grad(g_w.square().sum(), params + [x, wv], allow_unused=True)
        out.append((g_w.float(), [g if g is None else g.float() for g in g2]))
    tol = {torch.float16: 2e-2, torch.bfloat16: 5e-2, torch.float32: 1e-4}[dtype]
    # the fused VJP node (_LayerVJP) against the unfused layer, and against the fused layer's composed VJP
    for (gw1, g21), (gw2, g22) in [(out[0], out[1]), (out[0], out[2])]:
        assert rel_err(gw1, gw2) < tol
        for a_, b_ in zip(g21, g22):
            if b_ is None:
                continue
            assert a_ is not None
            assert rel_err(a_, b_) < 4 * tol


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(4, 32, 16, 16, 48), (2, 64, 32, 32, 64), (2, 512, 16, 16, 256)])
def test_fused_synthesis_layer_fast_backward(dtype, shape):
    """First-order backward through sg2_layer_bwd + dgrad(dot epilogue) + scaled wgrad vs the composed
    differentiable backward of the same fused forward: every parameter and input gradient."""
    from training import networks_stylegan2 as net
    from torch_utils.ops import modconv
    N, Cin, H, W, Cout = shape
    torch.manual_seed(11)
    layer = net.SynthesisLayer(Cin, Cout, w_dim=16, resolution=H, conv_clamp=256).to(DEV)
    with torch.no_grad():
        layer.noise_strength.fill_(0.3)
        layer.bias.copy_(torch.randn(Cout) * 0.2)
    x0 = torch.randn(N, Cin, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    w0 = torch.randn(N, 16, device=DEV)
    noise = torch.randn(N, 1, H, W, device=DEV)
    dy = torch.randn(N, Cout, H, W, device=DEV)
    params = [layer.weight, layer.bias, layer.noise_strength, layer.affine.weight, layer.affine.bias]
    res = []
    # fast (fused kernels), composed (differentiable primitives), f32 reference (composed, fp32 activations)
    for fast, dt in [(True, dtype), (False, dtype), (False, torch.float32)]:
        modconv.fast_backward = fast
        x = x0.clone().to(dt).requires_grad_(True)
        wv = w0.clone().requires_grad_(True)
        orig = torch.randn
        torch.randn = lambda *a, **k: noise.clone()
        try:
            y = layer(x, wv)
        finally:
            torch.randn = orig
        grads = torch.autograd.grad((y.float() * dy).sum(), [x, wv] + params)
        res.append([g.float() for g in grads])
    modconv.fast_backward = True
    tol = 1e-2 if dtype == torch.float16 else 4e-2
    for a_, b_, r_ in zip(*res):
        # the fused path keeps dz in f32 where the composed one rounds it to 16 bits: it may only be closer
        assert rel_err(a_, r_) < max(tol, 1.25 * rel_err(b_, r_))


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(2, 16, 24, 8), (3, 64, 7, 512), (1, 1024, 2, 64)])
def test_layer_bwd(dtype, shape):
    from torch_utils.ops import conv2d_gradfix as cg
    N, H, W, C = shape
    torch.manual_seed(3)
    y = (torch.randn(N, C, H, W, device=DEV) * 2).to(dtype).contiguous(memory_format=torch.channels_last)
    c = torch.randn(N, C, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, C, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    d = torch.rand(N, C, device=DEV) + 0.5
    dc, db, dd, dn = cg.layer_bwd(dy, y, c, d, act=1, alpha=0.2, gain=1.5, clamp=2.5)
    yf = y.float()
    dz = dy.float() * 1.5 * torch.where(yf > 0, 1.0, 0.2) * ((yf > -2.5) & (yf < 2.5)).float()
    tol = 5e-3 if dtype == torch.float16 else 2e-2
    assert rel_err(dc.float(), dz * d[:, :, None, None]) < tol
    assert rel_err(db, dz.sum([0, 2, 3])) < 1e-4
    assert rel_err(dd, (dz * c.float()).sum([2, 3])) < 1e-4
    assert rel_err(dn, dz.sum(1, keepdim=True)) < 1e-4


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(2, 64, 20, 33, 96), (9, 64, 128, 256, 64)])   # generic / persistent c64
def test_conv3x3_dot_and_scaled_wgrad(dtype, shape):
    from torch_utils.ops import conv2d_gradfix as cg
    torch.manual_seed(4)
    N, Cin, H, W, Cout = shape
    x = torch.randn(N, Cin, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, 3, 3, device=DEV) / np.sqrt(Cin * 9)).to(dtype)
    src = torch.randn(N, Cout, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    s = torch.rand(N, Cout, device=DEV) + 0.5
    y, raw, dot = cg.conv3x3_fused(x, cg._pack_conv(w), Cout, out_scale=s, dot_src=src)
    c = F.conv2d(x.double(), w.double(), padding=1)
    tol = 5e-3 if dtype == torch.float16 else 2e-2
    assert rel_err(y.float(), c * s[:, :, None, None].double()) < tol
    assert rel_err(dot, (c.to(dtype).double() * src.double()).sum([2, 3])) < tol
    g = torch.randn(N, Cout, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    xs = torch.rand(N, Cin, device=DEV) + 0.5
    dw = cg._wgrad_raw(g, x, 3, 3, 1, (1, 1), x_scale=xs)
    xsc = (x.float() * xs[:, :, None, None]).to(dtype)
    ref = torch.nn.grad.conv2d_weight(xsc.double(), w.shape, g.double(), padding=1)
    assert rel_err(dw, ref) < tol


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('r1_pass', [False, True])
def test_fused_d_conv_layer_matches_composed(dtype, r1_pass):
    """Discriminator 3x3 Conv2dLayer (bias + lrelu + clamp) through one sg2_conv3x3 launch and the fused
    backward vs the composed path (conv kernel + bias_act kernel): output, input/param grads and the
    R1-style second-order grads.  r1_pass: the create_graph gradient under no_weight_gradients, as loss.py's
    R1 term runs it (reference loss.py:125), which takes the fused VJP node (modconv._LayerVJP)."""
    import contextlib
    from training import networks_stylegan2 as net
    from torch_utils.ops import conv2d_gradfix, modconv
    ctx = conv2d_gradfix.no_weight_gradients if r1_pass else contextlib.nullcontext
    torch.manual_seed(13)
    layer = net.Conv2dLayer(32, 48, kernel_size=3, activation='lrelu', conv_clamp=256).to(DEV)
    with torch.no_grad():
        layer.bias.copy_(torch.randn(48) * 0.2)
    x0 = torch.randn(4, 32, 24, 16, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(4, 48, 24, 16, device=DEV)
    params = [layer.weight, layer.bias]
    res = []
    for fused in [True, False]:
        modconv.enabled = fused
        x = x0.clone().requires_grad_(True)
        y = layer(x, gain=np.sqrt(0.5))
        with ctx():
            gx, = torch.autograd.grad((y.float() * dy).sum(), [x], create_graph=True)
        g2 = torch.autograd.grad(gx.float().square().sum(), params)
        y = layer(x)
        g1 = torch.autograd.grad((y.float() * dy).sum(), [x] + params)
        res.append([y.float(), gx.float()] + [g.float() for g in g1] + [g.float() for g in g2])
    modconv.enabled = True
    tol = 1e-2 if dtype == torch.float16 else 4e-2
    for a_, b_ in zip(*res):
        assert rel_err(a_, b_) < tol


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(2, 64, 64, 32, 32), (3, 128, 96, 20, 37), (1, 512, 512, 32, 32), (2, 8, 40, 16, 16),
                                   (2, 72, 64, 17, 48)])
@pytest.mark.parametrize('scaled', [False, True])
def test_wgrad3x3_halo(dtype, shape, scaled):
    """sg2_conv2d_wgrad on the 3x3/s1/p1 halo path (all nine taps per tile) vs an f64 reference."""
    from torch_utils.ops import conv2d_gradfix as cg
    N, A, B, H, W = shape
    torch.manual_seed(21)
    g = torch.randn(N, A, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    x = torch.randn(N, B, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    s = (torch.rand(N, B, device=DEV) + 0.5) if scaled else None
    dw = cg._wgrad_raw(g, x, 3, 3, 1, (1, 1), x_scale=s)
    xs = (x.float() * s[:, :, None, None]).to(dtype) if scaled else x
    ref = torch.nn.grad.conv2d_weight(xs.double(), [A, B, 3, 3], g.double(), padding=1)
    assert rel_err(dw, ref) < (2e-3 if dtype == torch.float16 else 1e-2)


def _layer_grads(fwd, params, x0, dy, second_order):
    """Output, first-order grads (input + params) and, optionally, PL-style second-order grads."""
    x = x0.clone().requires_grad_(True)
    y = fwd(x)
    out = [y.float()]
    if second_order:
        gx, = torch.autograd.grad((y.float() * dy).sum(), [x], create_graph=True)
        g2 = torch.autograd.grad(gx.float().square().sum(), params, allow_unused=True)
        # a parameter outside the second-order graph (e.g. a bias under lrelu) has a zero gradient
        out += [(g if g is not None else torch.zeros_like(p_)).float() for g, p_ in zip(g2, params)]
        x = x0.clone().requires_grad_(True)
        y = fwd(x)
    out += [g.float() for g in torch.autograd.grad((y.float() * dy).sum(), [x] + params)]
    return out


def _fused_vs_composed(fwd, params, x0, dy, dtype, second_order=True, fwd32=None):
    """Fused vs composed path.  For 16-bit layers both are also compared with the composed path run in
    f32 (fwd32, or fwd on x0.float()): sums with heavy cancellation (e.g. the noise-strength gradient)
    carry the 16-bit rounding of the composed path, so the fused path must be within tolerance of the
    composed one OR no further from the f32 result than the composed path is."""
    from torch_utils.ops import modconv
    res = []
    for fused in [True, False]:
        modconv.enabled = fused
        try:
            res.append(_layer_grads(fwd, params, x0, dy, second_order))
        finally:
            modconv.enabled = True
    tol = {torch.float32: 1e-4, torch.float16: 1e-2, torch.bfloat16: 4e-2}[dtype]
    ref = None
    if dtype != torch.float32:
        modconv.enabled = False
        try:
            ref = _layer_grads(fwd32 or fwd, params, x0.float(), dy, second_order)
        finally:
            modconv.enabled = True
    assert len(res[0]) == len(res[1])
    for k, (a_, b_) in enumerate(zip(*res)):
        t = tol if k == 0 else 2 * tol
        if ref is None:
            assert rel_err(a_, b_) < t, k
        else:
            assert rel_err(a_, b_) < t or rel_err(a_, ref[k]) <= 1.25 * rel_err(b_, ref[k]) + 1e-3, k


@pytest.mark.parametrize('dtype', [torch.float32, torch.float16, torch.bfloat16])
def test_fused_up_synthesis_layer(dtype):
    """Up-2 SynthesisLayer: conv_transpose with the modulation in its operand staging + FIR with the
    demod/noise/bias/lrelu/clamp epilogue (UpModConv) vs the composed reference path."""
    from training import networks_stylegan2 as net
    torch.manual_seed(17)
    layer = net.SynthesisLayer(32, 48, w_dim=16, resolution=32, up=2, conv_clamp=256).to(DEV)
    with torch.no_grad():
        layer.noise_strength.fill_(0.3)
        layer.bias.copy_(torch.randn(48) * 0.2)
    x0 = torch.randn(4, 32, 16, 16, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    wv = torch.randn(4, 16, device=DEV)
    dy = 0.1 * (torch.randn(4, 48, 32, 32, device=DEV) + 0.5)   # positive-mean dy and |noise|: the noise-strength
    params = [layer.weight, layer.bias, layer.noise_strength, layer.affine.weight]   # gradient is then
    noise = torch.randn(4, 1, 32, 32, device=DEV).abs()    # well conditioned

    def fwd(x):
        orig = torch.randn
        torch.randn = lambda *a, **k: noise.clone()
        try:
            return layer(x, wv)
        finally:
            torch.randn = orig
    _fused_vs_composed(fwd, params, x0, dy, dtype)


@pytest.mark.parametrize('dtype', [torch.float32, torch.float16, torch.bfloat16])
def test_fused_discriminator_block(dtype):
    """Resnet DiscriminatorBlock: skip (FIR-down + 1x1, gain epilogue), conv0 and conv1 (FIR + stride-2
    conv with bias/lrelu/clamp epilogue and the skip added in the epilogue) vs the composed path."""
    from training import networks_stylegan2 as net
    torch.manual_seed(19)
    blk = net.DiscriminatorBlock(32, 32, 64, resolution=32, img_channels=1, first_layer_idx=0, conv_clamp=256,
                                 use_fp16=(dtype != torch.float32), fp16_dtype=dtype if dtype != torch.float32 else torch.float16).to(DEV)
    with torch.no_grad():
        for m in [blk.conv0, blk.conv1]:
            m.bias.copy_(torch.randn_like(m.bias) * 0.2)
    x0 = torch.randn(4, 32, 32, 32, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(4, 64, 16, 16, device=DEV)
    params = [blk.conv0.weight, blk.conv1.weight, blk.conv1.bias, blk.skip.weight]
    _fused_vs_composed(lambda x: blk(x, None)[0], params, x0, dy, dtype,
                       fwd32=lambda x: blk(x, None, force_fp32=True)[0])


@pytest.mark.parametrize('dtype', [torch.float32, torch.float16])
def test_fused_torgb_and_f32_layer(dtype):
    from training import networks_stylegan2 as net
    torch.manual_seed(23)
    torgb = net.ToRGBLayer(32, 1, w_dim=16, conv_clamp=256).to(DEV)
    with torch.no_grad():
        torgb.bias.fill_(0.1)
    x0 = torch.randn(4, 32, 16, 16, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    wv = torch.randn(4, 16, device=DEV)
    dy = torch.randn(4, 1, 16, 16, device=DEV)
    _fused_vs_composed(lambda x: torgb(x, wv), [torgb.weight, torgb.bias, torgb.affine.weight], x0, dy, dtype)
    layer = net.SynthesisLayer(32, 32, w_dim=16, resolution=8, conv_clamp=256).to(DEV)
    with torch.no_grad():
        layer.noise_strength.fill_(0.3)
    x1 = torch.randn(4, 32, 8, 8, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    dy1 = torch.randn(4, 32, 8, 8, device=DEV)
    _fused_vs_composed(lambda x: layer(x, wv, noise_mode='const'), [layer.weight, layer.bias, layer.noise_strength,
                                                                    layer.affine.weight], x1, dy1, dtype)


@pytest.mark.parametrize('fp16', [False, True])
def test_torgb_tap_matches_autograd_sum(fp16, monkeypatch):
    """SynthesisBlock feature maps feed both the toRGB layer and the next block: with modconv.FusedConvTap the two
    gradients of the map are added inside the toRGB input gradient's epilogue.  A whole small generator's first-order
    gradients (every parameter, and the latent input's) are bitwise those of autograd's own add (tap off), and the
    create_graph pass (the path-length shape: input gradients, then a second backward) matches to the rounding of
    a different summation order."""
    from training import networks_stylegan2 as net
    from torch_utils.ops import modconv
    torch.manual_seed(31)
    G = net.Generator(z_dim=32, c_dim=0, w_dim=32, img_resolution=64, img_channels=1, channel_base=2048,
                      channel_max=64, num_fp16_res=4 if fp16 else 0, conv_clamp=256,
                      mapping_kwargs=dict(num_layers=2)).to(DEV)
    z = torch.randn(4, 32, device=DEV)
    dy = torch.randn(4, 1, 64, 64, device=DEV)

    def grads(tap, second=False):
        monkeypatch.setattr(modconv, 'tap_enabled', tap)
        ws = G.mapping(z, None).detach().requires_grad_(True)
        img = G.synthesis(ws, noise_mode='const')
        if not second:
            gs = torch.autograd.grad((img * dy).sum(), [ws] + list(G.parameters()), allow_unused=True)
        else:
            g, = torch.autograd.grad((img * dy).sum(), [ws], create_graph=True)
            gs = torch.autograd.grad(g.square().sum(), [ws] + list(G.synthesis.parameters()), allow_unused=True)
        return [t for t in gs]
    import sg2hip
    for second in (False, True):
        with sg2hip.deterministic():        # fixed-order reductions: the comparison is of the tap alone
            a, b = grads(True, second), grads(False, second)
        for i, (u, v) in enumerate(zip(a, b)):
            assert (u is None) == (v is None), i
            if u is not None and not second:
                assert torch.equal(u, v), (i, float((u - v).abs().max()))
        if second:
            # the tap changes the order autograd runs the first pass's nodes in, so tensors with three or more
            # gradient contributions sum them in another order: the second pass differs by that rounding (the
            # deterministic baseline against itself is bitwise; tools/tap_diag.py) -- per tensor up to 3e-4 at 16
            # bits, more on the near-cancelling scalar noise-strength sums; judged on the whole flat gradient
            fa = torch.cat([u.float().flatten() for u in a if u is not None])
            fb = torch.cat([v.float().flatten() for v in b if v is not None])
            ok = torch.isfinite(fb)
            assert torch.equal(torch.isfinite(fa), ok)          # (a 16-bit second order can overflow: both alike)
            rel = float((fa[ok] - fb[ok]).norm() / fb[ok].norm())
            assert rel < (1e-3 if fp16 else 1e-5), rel


@pytest.mark.parametrize('dtype', [torch.float32, torch.float16])
@pytest.mark.parametrize('geom', [(3, 2, 0, True), (3, 2, 0, False), (3, 1, 1, False), (1, 1, 0, False),
                                  (1, 1, 0, True, 1, 64, 67, 61), (1, 1, 0, True, 3, 128, 9, 7),
                                  (1, 1, 0, False, 2, 512, 16, 16)])
def test_conv_fused_dot_and_scale(dtype, geom):
    """sg2_conv2d_fused: out_scale epilogue + per-(n, o) dot reduction against dot_src (the modulation
    gradient of a dgrad), for plain / strided / transposed geometries; Cin <= 4 runs the 1x1 outer-product
    kernel with its per-sample dot reduction (toRGB's input gradient), with pixel counts that leave the
    last workgroup of each sample partly empty."""
    from torch_utils.ops import conv2d_gradfix as cg
    k, stride, pad, transpose = geom[:4]
    torch.manual_seed(29)
    N, Cin, Cout, H, W = 3, 32, 48, 12, 10
    if len(geom) > 4:
        Cin, Cout, H, W = geom[4:]
    x = torch.randn(N, Cin, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    if transpose:
        w = (torch.randn(Cin, Cout, k, k, device=DEV) / (Cin * k * k) ** 0.5).to(dtype)
        ref = F.conv_transpose2d(x.double(), w.double(), stride=stride, padding=pad)
        wp = cg._pack_convT(w)
    else:
        w = (torch.randn(Cout, Cin, k, k, device=DEV) / (Cin * k * k) ** 0.5).to(dtype)
        ref = F.conv2d(x.double(), w.double(), stride=stride, padding=pad)
        wp = cg._pack_conv(w)
    oh, ow = ref.shape[2], ref.shape[3]
    s = torch.rand(N, Cout, device=DEV) + 0.5
    src = torch.randn(N, Cout, oh, ow, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    y, _, dot = cg.conv_fused(x, wp, Cout, oh, ow, k, k, stride, (pad, pad), transpose=transpose, out_scale=s,
                              dot_src=src)
    tol = 1e-5 if dtype == torch.float32 else 5e-3
    assert rel_err(y.float(), ref * s.double()[:, :, None, None]) < tol
    assert rel_err(dot, (ref.to(dtype).double() * src.double()).sum([2, 3])) < (1e-5 if dtype == torch.float32 else 5e-3)


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('case', ['conv_s2', 'convT_s2', 'conv_1x1', 'conv_s2_big', 'conv_s2_wide'])
@pytest.mark.parametrize('s2p', ['1', '0'])
def test_wgrad_halo_phases(dtype, case, s2p, monkeypatch):
    """Halo weight gradients: stride-2 conv (D down layers; all nine taps in one launch: the pipelined 16 x 6
    form wgrad3x3_s2p_kernel, s2p '0' the 16 x 8 wgrad3x3_s2_kernel), the transposed stride-2 conv of the up
    layers (with the modulation on the g operand) and 1x1 (phase kernel), vs autograd in f64; ragged tiles,
    partial 64-channel blocks, several tiles per workgroup (conv_s2_wide), in float-atomic and deterministic mode."""
    import sg2hip
    from torch_utils.ops import conv2d_gradfix as cg
    monkeypatch.setenv('SG2_WGRAD_S2P', s2p)
    torch.manual_seed(31)
    if case == 'conv_s2_wide':
        N, Ci, Co = 6, 64, 128
        x = torch.randn(N, Ci, 129, 97, device=DEV)
        w = torch.randn(Co, Ci, 3, 3, device=DEV, dtype=torch.float64, requires_grad=True)
        y = F.conv2d(x.to(dtype).double(), w, stride=2)
        g = torch.randn_like(y)
        ref, = torch.autograd.grad((y * g.to(dtype).double()).sum(), [w])
        for det in (False, True):
            with sg2hip.deterministic(det, device=DEV):
                dw = cg._wgrad_raw(g.to(dtype).contiguous(memory_format=torch.channels_last),
                                   x.to(dtype).contiguous(memory_format=torch.channels_last), 3, 3, 2, (0, 0))
            assert rel_err(dw, ref) < (2e-3 if dtype == torch.float16 else 1e-2)
        return
    N, Ci, Co = 2, 64, 72
    if case == 'conv_s2_big':
        N, Ci, Co = 3, 136, 64
        x = torch.randn(N, Ci, 67, 65, device=DEV)
        s = torch.rand(N, Ci, device=DEV) + 0.5
        w = torch.randn(Co, Ci, 3, 3, device=DEV, dtype=torch.float64, requires_grad=True)
        xs = (x.to(dtype).float() * s[:, :, None, None]).to(dtype).double()
        y = F.conv2d(xs, w, stride=2)
        g = torch.randn_like(y)
        ref, = torch.autograd.grad((y * g.to(dtype).double()).sum(), [w])
        dw = cg._wgrad_raw(g.to(dtype).contiguous(memory_format=torch.channels_last),
                           x.to(dtype).contiguous(memory_format=torch.channels_last), 3, 3, 2, (0, 0), x_scale=s)
    elif case == 'conv_s2':
        x = torch.randn(N, Ci, 33, 41, device=DEV)
        w = torch.randn(Co, Ci, 3, 3, device=DEV, dtype=torch.float64, requires_grad=True)
        y = F.conv2d(x.to(dtype).double(), w, stride=2)
        g = torch.randn_like(y)
        ref, = torch.autograd.grad((y * g.to(dtype).double()).sum(), [w])
        dw = cg._wgrad_raw(g.to(dtype).contiguous(memory_format=torch.channels_last),
                           x.to(dtype).contiguous(memory_format=torch.channels_last), 3, 3, 2, (0, 0))
    elif case == 'convT_s2':
        x = torch.randn(N, Ci, 16, 20, device=DEV)
        s = torch.rand(N, Ci, device=DEV) + 0.5
        wt = torch.randn(Ci, Co, 3, 3, device=DEV, dtype=torch.float64, requires_grad=True)
        xs = (x.to(dtype).float() * s[:, :, None, None]).to(dtype).double()
        y = F.conv_transpose2d(xs, wt, stride=2)
        dt = torch.randn_like(y)
        ref, = torch.autograd.grad((y * dt.to(dtype).double()).sum(), [wt])
        dw = cg._wgrad_raw(x.to(dtype).contiguous(memory_format=torch.channels_last),
                           dt.to(dtype).contiguous(memory_format=torch.channels_last), 3, 3, 2, (0, 0), g_scale=s)
    else:
        x = torch.randn(N, Ci, 24, 20, device=DEV)
        w = torch.randn(Co, Ci, 1, 1, device=DEV, dtype=torch.float64, requires_grad=True)
        y = F.conv2d(x.to(dtype).double(), w)
        g = torch.randn_like(y)
        ref, = torch.autograd.grad((y * g.to(dtype).double()).sum(), [w])
        dw = cg._wgrad_raw(g.to(dtype).contiguous(memory_format=torch.channels_last),
                           x.to(dtype).contiguous(memory_format=torch.channels_last), 1, 1, 1, (0, 0))
    assert rel_err(dw, ref) < (2e-3 if dtype == torch.float16 else 1e-2)


@pytest.mark.parametrize('dp', [0.02, 0.5, 0.97])
def test_augment_dynamic_extent(dp):
    """ADA geometric pipe at 128^2, 2 channels: the padded image is dynamically sized inside static buffers
    and the up-sampling passes / their adjoints / the grid-sample gradient only touch its extent
    (upfirdn2d.upsample2d_limited, sg2_upfirdn2d_lim).  Forward, input gradient and the R1-style double
    backward vs the CPU oracle (debug_percentile: deterministic transforms, small and large margins)."""
    from training import augment_mi
    cfg = dict(xflip=1, rotate90=1, xint=1, scale=1, rotate=1, aniso=1, xfrac=1)
    torch.manual_seed(5)
    x = torch.randn(3, 2, 128, 128)
    dy = torch.randn(3, 2, 128, 128)
    res = []
    for dev, pipe in [(DEV, augment_mi.AugmentPipe(run_dir=None, batch_size=3, **cfg).to(DEV)),
                      (torch.device('cpu'), O.AugmentPipe(**cfg))]:
        xd = x.to(dev).requires_grad_(True)
        y = pipe(xd, False, debug_percentile=dp)
        g, = torch.autograd.grad((y * y).sum(), [xd], create_graph=True)       # 2 A^T A x
        gg, = torch.autograd.grad((g * dy.to(dev)).sum(), [xd])                 # 2 A^T A dy
        res.append([t.detach().double().cpu() for t in (y, g, gg)])
    for a, b in zip(*res):
        assert rel_err(a, b) < 2e-5


def test_demod_kernel():
    """sg2_demod_fwd / sg2_demod_bwd (networks_stylegan2._Demod) vs autograd of the reference expression
    (networks_stylegan2.py:59-63) in fp64: value, first-order gradients and a create_graph second order."""
    from training import networks_stylegan2 as net
    torch.manual_seed(41)
    w = torch.randn(96, 80, 3, 3, device=DEV)
    s = torch.rand(5, 80, device=DEV) + 0.2
    dd = torch.randn(5, 96, device=DEV)
    ref = []
    for dev, fn in [(DEV, net._Demod.apply),
                    (torch.device('cpu'), lambda w_, s_: ((w_[None] * s_[:, None, :, None, None]).square()
                                                          .sum([2, 3, 4]) + 1e-8).rsqrt())]:
        dt = torch.float32 if dev.type == 'cuda' else torch.float64
        wd = w.to(dev, dt).requires_grad_(True)
        sd = s.to(dev, dt).requires_grad_(True)
        d = fn(wd, sd)
        gw, gs = torch.autograd.grad((d * dd.to(dev, dt)).sum(), [wd, sd], create_graph=True)
        gw2, = torch.autograd.grad((gs.square().sum() + gw.square().sum()), [wd])
        gwf, gsf = torch.autograd.grad((fn(wd, sd) * dd.to(dev, dt)).sum(), [wd, sd])   # first-order kernel path
        # the path-length shape (_DemodVJP): first pass for the styles only under no_weight_gradients, then a
        # second pass into both the weight and the styles through that gradient and through d itself
        from torch_utils.ops import conv2d_gradfix as cg
        dp = fn(wd, sd)
        with cg.no_weight_gradients(dev.type == 'cuda'):
            gsp, = torch.autograd.grad((dp * dd.to(dev, dt)).sum(), [sd], create_graph=True)
        gw3, gs3 = torch.autograd.grad(gsp.square().sum() + (dp * dd.to(dev, dt)).square().sum(), [wd, sd])
        ref.append([t.detach().double().cpu() for t in (d, gw, gs, gw2, gwf, gsf, gsp, gw3, gs3)])
    for a, b in zip(*ref):
        assert rel_err(a, b) < 1e-5


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('cin,cout', [(1, 64), (3, 16), (64, 1), (128, 3)])
def test_conv1x1_small_depth(dtype, cin, cout):
    """1x1 convolutions with <= 4 channels on one side (conv1x1_smallk / conv1x1_smallo, and the
    1x1 weight gradients wgrad1x1_small{a,b}): modulation, the full epilogue (out_scale, noise, bias,
    lrelu, gain, clamp, aux, residual) and the scaled weight gradient vs fp64."""
    from torch_utils.ops import conv2d_gradfix as cg
    torch.manual_seed(11)
    n, h, w = 2, 9, 13
    tol = {torch.float16: 3e-3, torch.bfloat16: 2e-2}[dtype]
    x = torch.randn(n, cin, h, w).to(dtype)
    wt = (torch.randn(cout, cin, 1, 1) / cin ** 0.5).to(dtype)
    s_in = torch.rand(n, cin) + 0.5
    s_out = torch.rand(n, cout) + 0.5
    noise = torch.randn(n, h, w).to(dtype)
    bias = torch.randn(cout).to(dtype).float()
    res = torch.randn(n, cout, h, w).to(dtype)
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    for aux_mode in (1, 2):
        y, aux = cg.conv_fused(xd, cg._pack_conv(wt.to(DEV)), cout, h, w, 1, 1, 1, (0, 0), in_scale=s_in.to(DEV),
                               out_scale=s_out.to(DEV), noise=noise.to(DEV), noise_gain=0.3, bias=bias.to(DEV), act=1,
                               alpha=0.2, gain=1.4, clamp=2.5, residual=res.to(DEV), aux_mode=aux_mode)
        xs = (x.float() * s_in[:, :, None, None]).to(dtype).double()          # operand rounded as in the kernels
        c = F.conv2d(xs, wt.double())
        z = c * s_out[:, :, None, None].double() + noise[:, None].double() * 0.3 + bias[None, :, None, None].double()
        z = (torch.where(z > 0, z, z * 0.2) * 1.4).clamp(-2.5, 2.5)
        assert rel_err(aux.float(), c if aux_mode == 1 else z) < tol, (cin, cout, aux_mode)
        assert rel_err(y.float(), z.to(dtype).double() + res.double()) < tol, (cin, cout, aux_mode)
    # weight gradient of the 1x1 conv with both operands modulated
    g = torch.randn(n, cout, h, w).to(dtype)
    gs, xsc = torch.rand(n, cout) + 0.5, torch.rand(n, cin) + 0.5
    dw = cg._wgrad_raw(g.to(DEV).contiguous(memory_format=torch.channels_last), xd, 1, 1, 1, (0, 0),
                       x_scale=xsc.to(DEV), g_scale=gs.to(DEV))
    ga = (g.float() * gs[:, :, None, None]).to(dtype).double()
    xa = (x.float() * xsc[:, :, None, None]).to(dtype).double()
    ref = torch.einsum('nahw,nbhw->ab', ga, xa)[:, :, None, None]
    assert rel_err(dw.cpu(), ref) < 1e-4, (cin, cout)


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
def test_dot_hw(dtype):
    """sg2_dot_hw (sum over pixels of a rounded 16-bit product, f32 accumulation) and its differentiable
    wrapper vs the composed (a * b).sum([2, 3], dtype=float32): value, gradient, double backward."""
    from torch_utils.ops import conv2d_gradfix as cg
    torch.manual_seed(5)
    a = torch.randn(3, 64, 11, 17, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    b = torch.randn(3, 64, 11, 17, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    a1, b1 = a.clone().requires_grad_(True), b.clone().requires_grad_(True)
    a2, b2 = a.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y1 = cg.dot_hw(a1, b1)
    y2 = (a2 * b2).sum([2, 3], dtype=torch.float32)
    assert rel_err(y1, y2.double().cpu()) < 1e-5
    g = torch.randn(3, 64, device=DEV)
    ga1, gb1 = torch.autograd.grad(y1, [a1, b1], g, create_graph=True)
    ga2, gb2 = torch.autograd.grad(y2, [a2, b2], g, create_graph=True)
    assert rel_err(ga1.float(), ga2.double().cpu()) < 1e-3 and rel_err(gb1.float(), gb2.double().cpu()) < 1e-3
    h1, = torch.autograd.grad((ga1.float() ** 2).sum(), [b1])
    h2, = torch.autograd.grad((ga2.float() ** 2).sum(), [b2])
    assert rel_err(h1.float(), h2.double().cpu()) < 1e-2


@pytest.mark.parametrize('src,dst', [(torch.float32, torch.float32), (torch.float32, torch.float16),
                                     (torch.float32, torch.bfloat16), (torch.float16, torch.float16)])
@pytest.mark.parametrize('o,i,k', [(512, 512, 3), (64, 1, 1), (3, 70, 3), (45, 33, 1), (96, 40, 3), (20, 37, 2),
                                   (6, 1000, 3)])
def test_pack_weight(src, dst, o, i, k):
    """sg2_pack_weight (conv2d_gradfix._pack_conv / _pack_convT, flipped taps, transposed views, ragged
    tiles) vs the torch permute-copy it replaces: bit-exact (a layout move plus one rounding).  Rows of B x K <=
    8192 take the row-mode kernel (misc.hip PACK_ROW_MAX), (6, 1000, 3)'s transposed packs the element mode."""
    from torch_utils.ops import conv2d_gradfix as cg
    torch.manual_seed(7)
    w = torch.randn(o, i, k, k, device=DEV).to(src)
    cases = [(cg._pack_conv(w, dst), w.permute(0, 2, 3, 1)),
             (cg._pack_convT(w, dst), w.permute(1, 2, 3, 0)),
             (cg._pack_convT(w, dst, flip=True), w.flip([2, 3]).permute(1, 2, 3, 0)),
             (cg._pack_conv(w, dst, flip=True), w.flip([2, 3]).permute(0, 2, 3, 1)),
             (cg._pack_conv(w.transpose(0, 1), dst), w.transpose(0, 1).permute(0, 2, 3, 1))]
    for got, ref in cases:
        ref = ref.to(dst).contiguous()
        assert got.shape == ref.shape and got.dtype == dst and got.is_contiguous()
        assert torch.equal(got, ref)


def test_infnorm_prenorm():
    """sg2_infnorm_fwd / _bwd (networks_stylegan2._prenorm, the fp16 pre-normalisation of :52-54) vs the
    reference expression under torch autograd: forward bit-exact; first-order gradients (with tied and
    negative maxima) and a create_graph second order to 1e-6."""
    from training import networks_stylegan2 as net
    torch.manual_seed(5)
    w = torch.randn(48, 40, 3, 3, device=DEV)
    w[3, 5, 1, 1] = w[3].abs().max() + 1.0          # a tie: two entries of equal magnitude, opposite sign
    w[3, 7, 0, 2] = -w[3, 5, 1, 1]
    w[9, 0, 0, 0] = -(w[9].abs().max() + 0.5)       # negative maximum
    s = torch.randn(6, 40, device=DEV)
    s[2, 4] = s[2, 11] = s[2].abs().max() + 0.25
    gy_w, gy_s = torch.randn_like(w), torch.randn_like(s)

    def ref(w_, s_):
        return (w_ * (1 / np.sqrt(40 * 9) / w_.norm(float('inf'), dim=[1, 2, 3], keepdim=True)),
                s_ / s_.norm(float('inf'), dim=1, keepdim=True))

    out = []
    for fn in (net._prenorm, ref):
        wd, sd = w.clone().requires_grad_(True), s.clone().requires_grad_(True)
        yw, ys = fn(wd, sd)
        gw, gs = torch.autograd.grad((yw * gy_w).sum() + (ys * gy_s).sum(), [wd, sd])
        wd2, sd2 = w.clone().requires_grad_(True), s.clone().requires_grad_(True)
        yw2, ys2 = fn(wd2, sd2)
        g1w, g1s = torch.autograd.grad((yw2 * gy_w).sum() + (ys2 * gy_s).sum(), [wd2, sd2], create_graph=True)
        g2w, g2s = torch.autograd.grad((g1w * gy_w).sum() + (g1s * gy_s).sum() + (yw2.square()).sum(), [wd2, sd2])
        out.append([yw.detach(), ys.detach(), gw, gs, g1w.detach(), g1s.detach(), g2w, g2s])
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    for a, b in zip(out[0][2:], out[1][2:]):
        assert rel_err(a.double().cpu(), b.double().cpu()) < 1e-6


def test_infnorm_prenorm_nan_rows():
    """A NaN in a row makes that row's norm(inf) NaN (torch's amax propagates it) -- the fused reduction
    must not drop it as fmaxf would; forward and gradient NaN patterns match the reference expression and
    the finite rows are unaffected."""
    from training import networks_stylegan2 as net
    torch.manual_seed(6)
    w = torch.randn(8, 16, 3, 3, device=DEV)
    w[2, 3, 1, 0] = float('nan')
    s = torch.randn(4, 16, device=DEV)
    s[1, 7] = float('nan')
    gy_w, gy_s = torch.randn_like(w), torch.randn_like(s)

    def ref(w_, s_):
        return (w_ * (1 / np.sqrt(16 * 9) / w_.norm(float('inf'), dim=[1, 2, 3], keepdim=True)),
                s_ / s_.norm(float('inf'), dim=1, keepdim=True))

    out = []
    for fn in (net._prenorm, ref):
        wd, sd = w.clone().requires_grad_(True), s.clone().requires_grad_(True)
        yw, ys = fn(wd, sd)
        gw, gs = torch.autograd.grad((yw * gy_w).sum() + (ys * gy_s).sum(), [wd, sd])
        out.append([yw.detach(), ys.detach(), gw, gs])
    assert torch.isnan(out[0][0][2]).all() and torch.isnan(out[0][1][1]).all()
    for a, b in zip(out[0][:2], out[1][:2]):
        torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)
    for a, b in zip(out[0][2:], out[1][2:]):
        assert torch.equal(torch.isnan(a), torch.isnan(b))
        fin = ~torch.isnan(a)
        assert rel_err(a[fin].double().cpu(), b[fin].double().cpu()) < 1e-6


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16, torch.float32])
def test_pack_scale_and_wgrad_alpha(dtype):
    """The weight gain of a Conv2dLayer (`weight * weight_gain`, networks_stylegan2.py:173) folded into
    sg2_pack_weight (scale: bit-identical to the f32 product cast to the activation dtype) and into
    sg2_conv2d_wgrad (alpha: the weight gradient times the gain), on the halo, generic and 1x1 paths."""
    from torch_utils.ops import conv2d_gradfix as cg
    torch.manual_seed(21)
    gain = 1 / np.sqrt(64 * 9)
    w = torch.randn(48, 64, 3, 3, device=DEV)
    assert torch.equal(cg._pack_conv(w, dtype, scale=gain), cg._pack_conv((w * gain).to(dtype)))
    assert torch.equal(cg._pack_convT(w, dtype, flip=True, scale=gain), cg._pack_convT((w * gain).to(dtype), flip=True))
    for (n, a, b, h, k, s, p) in [(2, 48, 64, 20, 3, 1, 1), (2, 48, 64, 20, 3, 2, 0), (2, 40, 24, 9, 1, 1, 0)]:
        oh = (h + 2 * p - k) // s + 1
        g = torch.randn(n, a, oh, oh, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
        x = torch.randn(n, b, h, h, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
        ref = cg._wgrad_raw(g, x, k, k, s, (p, p)) * gain
        got = cg._wgrad_raw(g, x, k, k, s, (p, p), alpha=gain)
        assert rel_err(got, ref) < 1e-6, (n, a, b, h, k, s, p)


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(2, 128, 65, 70, 64), (2, 64, 64, 64, 128), (1, 512, 64, 64, 512), (1, 32, 64, 96, 8),
                                   (2, 64, 16, 16, 128), (2, 512, 32, 32, 256), (1, 64, 136, 272, 64),
                                   (1, 32, 16, 48, 64)])
@pytest.mark.parametrize('mod', [False, True])
def test_conv3x3_up2(dtype, shape, mod, monkeypatch):
    """sg2_conv3x3_up2 (the stride-2 transposed 3x3 conv of the up-2 layers, output 2H+1, with the
    modulation x * s.to(x.dtype) in its staging) vs F.conv_transpose2d in float64 on the same rounded
    operands; ragged tiles (H, W not multiples of the 8 x 16 cell tile), Cout below one 64-channel block; the
    edge split (16^2 and 32^2 inputs, several row / column strips at 136 x 272) bitwise against the ragged tiling."""
    from torch_utils.ops import conv2d_gradfix as cg
    N, Cin, H, W, Cout = shape
    torch.manual_seed(31)
    x = torch.randn(N, Cin, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, 3, 3, device=DEV) / np.sqrt(Cin * 9)).to(dtype)   # the modulated-conv layout
    s = (torch.rand(N, Cin, device=DEV) + 0.5) if mod else None
    assert cg._up2_ok(x, Cout, 2 * H + 1, 2 * W + 1, 3, 3, 2, (0, 0), True)
    y, _ = cg.conv_fused(x, cg._pack_conv(w), Cout, 2 * H + 1, 2 * W + 1, 3, 3, 2, (0, 0), transpose=True, in_scale=s)
    xs = (x.float() * s.to(dtype).float()[:, :, None, None]).to(dtype) if mod else x
    ref = F.conv_transpose2d(xs.double(), w.double().transpose(0, 1), stride=2)
    assert y.shape == ref.shape
    tol = 5e-3 if dtype == torch.float16 else 2e-2
    assert rel_err(y.float(), ref) < tol
    if H % 8 == 0 and W % 16 == 0:   # the edge split (last cell row / column as three-tap strips): the same sums
        monkeypatch.setenv('SG2_UP2_EDGE', '0')
        ys = cg._conv_up2(x, cg._pack_conv(w), Cout, in_scale=s)
        assert torch.equal(y, ys)


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(2, 64, 65, 65, 128), (2, 128, 69, 133, 64), (1, 512, 65, 65, 512),
                                   (2, 40, 67, 71, 8), (1, 64, 257, 257, 128), (2, 512, 33, 33, 512),
                                   (3, 256, 17, 19, 512)])
def test_conv3x3_s2(dtype, shape):
    """sg2_conv3x3_s2 (stride 2, pad 0: the discriminator's down-2 3x3 layers and the up-2 layers' input
    gradient) vs F.conv2d in float64 on the same rounded operands: the full layer epilogue with the raw
    output, the resnet residual with the pre-residual epilogue value, and the out_scale + dot form;
    ragged 32 x 4 output tiles, Cin = 40 (one partial K chunk), Cout below one block."""
    from torch_utils.ops import conv2d_gradfix as cg
    N, Cin, H, W, Cout = shape
    OH, OW = (H - 3) // 2 + 1, (W - 3) // 2 + 1
    torch.manual_seed(41)
    x = torch.randn(N, Cin, H, W)
    w = torch.randn(Cout, Cin, 3, 3) / np.sqrt(Cin * 9)
    s = torch.rand(N, Cin) + 0.5
    d = torch.rand(N, Cout) + 0.5
    noise = torch.randn(N, 1, OH, OW)
    b = torch.randn(Cout) * 0.1
    res = torch.randn(N, Cout, OH, OW)
    xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv(w.to(DEV, dtype))
    tol = 5e-3 if dtype == torch.float16 else 2e-2
    xs = (x.to(dtype).float() * s[:, :, None, None]).to(dtype).double()
    c = F.conv2d(xs, w.to(dtype).double(), stride=2)
    # (1) modulated conv + demod + noise + bias + lrelu + clamp, raw output
    y, raw = cg.conv3x3_fused(xd, wp, Cout, in_scale=s.to(DEV), out_scale=d.to(DEV),
                              noise=noise.to(DEV, dtype).reshape(N, OH, OW).contiguous(), noise_gain=0.3,
                              bias=b.to(DEV), act=1, alpha=0.2, gain=np.sqrt(2), clamp=1.5, want_raw=True, stride=2)
    z = c * d[:, :, None, None] + noise.to(dtype).double() * 0.3 + b[None, :, None, None]
    yr = (F.leaky_relu(z, 0.2) * np.sqrt(2)).clamp(-1.5, 1.5)
    assert y.shape == (N, Cout, OH, OW)
    assert rel_err(raw.float(), c) < tol
    assert rel_err(y.float(), yr) < tol
    # (2) bias + lrelu + residual (DiscriminatorBlock conv1), raw = the activation before the add
    rd = res.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    y, za = cg.conv3x3_fused(xd, wp, Cout, bias=b.to(DEV), act=1, alpha=0.2, gain=np.sqrt(0.5), clamp=256.0,
                             want_raw=True, stride=2, residual=rd, raw_act=True)
    c0 = F.conv2d(x.to(dtype).double(), w.to(dtype).double(), stride=2)
    zr = F.leaky_relu(c0 + b[None, :, None, None], 0.2) * np.sqrt(0.5)
    assert rel_err(za.float(), zr) < tol
    assert rel_err(y.float(), zr + res.to(dtype).double()) < tol
    assert torch.equal(y, (za.float() + rd.float()).to(dtype))     # round(z) + residual, rounded once more
    # (3) out_scale + dot (the up-2 layer's dgrad: dx and ds in one launch)
    src = torch.randn(N, Cout, OH, OW).to(dtype)
    y, _, dot = cg.conv3x3_fused(xd, wp, Cout, out_scale=d.to(DEV), dot_src=src.to(DEV).contiguous(
        memory_format=torch.channels_last), stride=2)
    cd = F.conv2d(x.to(dtype).double(), w.to(dtype).double(), stride=2)
    assert rel_err(y.float(), cd * d[:, :, None, None]) < tol
    assert rel_err(dot, (cd * src.double()).sum([2, 3])) < tol


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(2, 64, 129, 129, 128), (3, 128, 65, 65, 256), (1, 256, 65, 65, 512),
                                   (2, 32, 67, 67, 128), (1, 64, 257, 257, 128), (5, 96, 71, 65, 384)])
@pytest.mark.parametrize('s2g', ['1', '0'])
def test_conv3x3_s2g(dtype, shape, s2g, monkeypatch):
    """The wide stride-2 down layers on the LDS-DMA implicit GEMM (conv3x3.hip conv3x3_s2g_kernel; s2g '0': the
    32 x 4 halo form it replaces) vs F.conv2d in float64: plain, the D block's bias + lrelu + gain + clamp with the
    raw output, the resnet residual with the pre-residual activation, and a demodulation scale.  Shapes: several
    output-channel tiles (Cout 256 .. 512), a ragged last pixel tile (2 x 33 x 33 pixels), Cin = 32 (one K chunk a
    tap), non-square input."""
    from torch_utils.ops import conv2d_gradfix as cg
    monkeypatch.setenv('SG2_S2G', s2g)
    N, Cin, H, W, Cout = shape
    OH, OW = (H - 3) // 2 + 1, (W - 3) // 2 + 1
    assert cg._halo_s2_ok(torch.empty(N, Cin, H, W, dtype=dtype), 3, 3, 2, 0, cout=Cout)
    torch.manual_seed(43)
    x = torch.randn(N, Cin, H, W)
    w = torch.randn(Cout, Cin, 3, 3) / np.sqrt(Cin * 9)
    b = torch.randn(Cout) * 0.1
    d = torch.rand(N, Cout) + 0.5
    res = torch.randn(N, Cout, OH, OW)
    xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv(w.to(DEV, dtype))
    tol = 5e-3 if dtype == torch.float16 else 2e-2
    c = F.conv2d(x.to(dtype).double(), w.to(dtype).double(), stride=2)
    y, _ = cg.conv3x3_fused(xd, wp, Cout, stride=2)                       # plain
    assert y.shape == (N, Cout, OH, OW) and rel_err(y.float(), c) < tol
    for n in range(N):
        assert rel_err(y[n].float(), c[n]) < tol, n
    y, raw = cg.conv3x3_fused(xd, wp, Cout, bias=b.to(DEV), act=1, alpha=0.2, gain=np.sqrt(2), clamp=1.5,
                              want_raw=True, stride=2)
    assert rel_err(raw.float(), c) < tol
    assert rel_err(y.float(), (F.leaky_relu(c + b[None, :, None, None], 0.2) * np.sqrt(2)).clamp(-1.5, 1.5)) < tol
    rd = res.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    y, za = cg.conv3x3_fused(xd, wp, Cout, bias=b.to(DEV), act=1, alpha=0.2, gain=np.sqrt(0.5), clamp=256.0,
                             want_raw=True, stride=2, residual=rd, raw_act=True)
    zr = F.leaky_relu(c + b[None, :, None, None], 0.2) * np.sqrt(0.5)
    assert rel_err(za.float(), zr) < tol
    assert torch.equal(y, (za.float() + rd.float()).to(dtype))            # round(z) + residual, rounded once more
    y, raw = cg.conv3x3_fused(xd, wp, Cout, out_scale=d.to(DEV), want_raw=True, stride=2, residual=rd)
    assert rel_err(raw.float(), c) < tol
    assert rel_err(y.float(), c * d[:, :, None, None] + res.to(dtype).double()) < tol


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
def test_down_layer_s2_route_matches_generic(dtype, monkeypatch):
    """A discriminator down-2 Conv2dLayer with the resnet residual (networks_stylegan2.py:621-627) through
    the stride-2 halo kernel vs the same layer forced onto the generic implicit-GEMM kernel: output and
    first-order gradients (x, weight, bias, residual)."""
    from torch_utils.ops import conv2d_gradfix as cg
    from torch_utils.ops import modconv
    torch.manual_seed(43)
    N, Cin, H, Cout = 4, 64, 33, 128
    x0 = torch.randn(N, Cin, H, H, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    w0 = torch.randn(Cout, Cin, 3, 3, device=DEV)
    b0 = torch.randn(Cout, device=DEV) * 0.1
    r0 = torch.randn(N, Cout, 16, 16, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    g = torch.randn(N, Cout, 16, 16, device=DEV).to(dtype)
    assert cg._halo_s2_ok(x0, 3, 3, 2, (0, 0))

    def run():
        x, w, b, r = (t.detach().clone().requires_grad_(True) for t in (x0, w0, b0, r0))
        y = modconv.fused_conv(x, w.to(dtype), bias=b, residual=r, stride=2, padding=0, act='lrelu',
                               gain=np.sqrt(0.5), clamp=256.0, wgain=1 / np.sqrt(Cin * 9))
        y.backward(g)
        return [t.float() for t in (y, x.grad, w.grad, b.grad, r.grad)]

    fast = run()
    monkeypatch.setattr(cg, '_halo_s2_ok', lambda *a, **k: False)
    slow = run()
    tol = 5e-3 if dtype == torch.float16 else 2e-2
    for name, a_, b_ in zip(('y', 'dx', 'dw', 'db', 'dres'), fast, slow):
        assert rel_err(a_, b_) < tol, name


@pytest.mark.parametrize('dtype', [torch.float32, torch.float16])
def test_fork_fir_discriminator_block(dtype, monkeypatch):
    """DiscriminatorBlock with the skip's FIR forked off its input (upfirdn2d.fork_fir: the skip / conv0
    gradient add fused into the adjoint FIR's epilogue, rounding FIR^T(g) and the sum as the separate
    launches do) vs the plain two-branch graph: forward, first-order gradients and an R1-style double
    backward (create_graph) through both."""
    from torch_utils.ops import upfirdn2d as up
    from training import networks_stylegan2 as net
    torch.manual_seed(29)
    blk = net.DiscriminatorBlock(64, 64, 128, resolution=32, img_channels=1, first_layer_idx=0, conv_clamp=256,
                                 use_fp16=(dtype != torch.float32), fp16_dtype=torch.float16).to(DEV)
    x0 = torch.randn(4, 64, 32, 32, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(4, 128, 16, 16, device=DEV)
    params = [blk.conv0.weight, blk.conv1.weight, blk.skip.weight]

    def run():
        x = x0.detach().clone().requires_grad_(True)
        y = blk(x, None)[0]
        g = torch.autograd.grad(y, [x] + params, dy.to(y.dtype))
        x2 = x0.detach().clone().float().requires_grad_(True)
        y2 = blk(x2.to(dtype).contiguous(memory_format=torch.channels_last), None)[0]
        (gx,) = torch.autograd.grad(y2.float().square().sum(), [x2], create_graph=True)
        r1 = torch.autograd.grad(gx.square().sum(), params)
        return y, g, r1

    assert up.fork_fir_ok(x0, blk.skip.resample_filter)
    calls = []
    orig = up.fork_fir
    monkeypatch.setattr(up, 'fork_fir', lambda *a: calls.append(1) or orig(*a))
    y_f, g_f, r_f = run()
    assert calls
    monkeypatch.setattr(up, 'fork_fir_ok', lambda *a: False)
    y_p, g_p, r_p = run()
    # (not bitwise: the split-K convs of this small block accumulate with float atomics, so two runs of
    # either graph differ in the last bits)
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    assert rel_err(y_f.float(), y_p.float()) < tol
    for a_, b_ in zip(g_f, g_p):
        assert rel_err(a_.float(), b_.float()) < tol
    for a_, b_ in zip(r_f, r_p):
        assert rel_err(a_.float(), b_.float()) < 1e-3


def test_split_k_clean_workspace():
    """Split-K convs (f32 low-resolution layers) run on one persistent workspace that each call leaves zeroed
    (sg2_set_clean_workspace: no memset per call): repeated calls give the same result as a fresh-workspace
    call, and the workspace is all zeros afterwards."""
    from torch_utils.ops import conv2d_gradfix as cg
    torch.manual_seed(11)
    x = torch.randn(32, 512, 8, 8, device=DEV).contiguous(memory_format=torch.channels_last)
    w = torch.randn(512, 512, 3, 3, device=DEV) / 48
    wp = cg._pack_conv(w)
    first = cg._conv_raw(x, wp, 512, 8, 8, 3, 3, 1, (1, 1), False)
    assert x.device in cg._CLEAN_WS
    for _ in range(3):
        again = cg._conv_raw(x, wp, 512, 8, 8, 3, 3, 1, (1, 1), False)
        assert torch.equal(again, first) or rel_err(again, first) < 1e-6   # split-K atomics: order may vary
    torch.cuda.synchronize()
    assert float(cg._CLEAN_WS[x.device].abs().max()) == 0.0
    ref = torch.nn.functional.conv2d(x.double(), w.double(), padding=1)
    assert rel_err(first.double(), ref) < 1e-5
    # captured into a graph and replayed back to back with eager calls: the same shared workspace
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cap = cg._conv_raw(x, wp, 512, 8, 8, 3, 3, 1, (1, 1), False)
    for _ in range(2):
        g.replay()
        eager = cg._conv_raw(x, wp, 512, 8, 8, 3, 3, 1, (1, 1), False)
    torch.cuda.synchronize()
    assert rel_err(cap, first) < 1e-6 and rel_err(eager, first) < 1e-6
    assert float(cg._CLEAN_WS[x.device].abs().max()) == 0.0
    # a failing call drops the workspace (it may be dirty); the next call gets a fresh zeroed one
    ws0 = cg._CLEAN_WS[x.device]
    with pytest.raises(RuntimeError):
        with cg._split_k(x, True):
            raise RuntimeError('launch failed')
    assert x.device not in cg._CLEAN_WS
    again = cg._conv_raw(x, wp, 512, 8, 8, 3, 3, 1, (1, 1), False)
    assert cg._CLEAN_WS[x.device] is not ws0 and rel_err(again, first) < 1e-6


def test_depthwise_1d_grouped_conv():
    """conv2d(groups = C) with one channel per group and a 1 x K / K x 1 kernel (the ADA image filter:
    groups = N * C, per-sample taps) runs as K multiply-adds: forward, input / weight gradients and the
    double backward (R1 through the augment pipe) vs torch's fp64 grouped conv."""
    from torch_utils.ops import conv2d_gradfix as cg
    torch.manual_seed(7)
    for kshape in [(1, 12), (12, 1)]:
        x = torch.randn(1, 10, 30, 27, device=DEV, requires_grad=True)
        w = torch.randn(10, 1, *kshape, device=DEV, requires_grad=True)
        assert cg._depthwise_1d(x, w, 10, 1, 0, 0)
        y = cg.conv2d(x, w, groups=10)
        xr, wr = x.detach().double().requires_grad_(True), w.detach().double().requires_grad_(True)
        yr = torch.nn.functional.conv2d(xr, wr, groups=10)
        assert rel_err(y.double(), yr) < 1e-6
        dy = torch.randn_like(y)
        gx, gw = torch.autograd.grad((y * dy).sum(), [x, w], create_graph=True)
        gxr, gwr = torch.autograd.grad((yr * dy.double()).sum(), [xr, wr], create_graph=True)
        assert rel_err(gx.double(), gxr) < 1e-6 and rel_err(gw.double(), gwr) < 1e-6
        ggw, = torch.autograd.grad(gx.square().sum(), [w])
        ggwr, = torch.autograd.grad(gxr.square().sum(), [wr])
        assert rel_err(ggw.double(), ggwr) < 1e-5


@pytest.mark.parametrize('mode', ['composed', 'create_graph'])
def test_fused_conv_wgain_weight_grad(mode):
    """FusedConv with a weight gain (a Conv2dLayer's 1/sqrt(fan_in), networks_stylegan2.py:173) on the composed
    backward -- modconv.fast_backward off, or a create_graph backward -- vs float64 torch: the weight gradient is
    for the RAW weight, dL/dW = wgain * dL/d(W * wgain), as are dx and db (the composed path once
    returned dL/d(W * wgain))."""
    from torch_utils.ops import modconv
    torch.manual_seed(51)
    N, Cin, H, Cout = 2, 16, 12, 24
    wgain = 1 / np.sqrt(Cin * 9)
    x0 = torch.randn(N, Cin, H, H, device=DEV).contiguous(memory_format=torch.channels_last)
    w0 = torch.randn(Cout, Cin, 3, 3, device=DEV)
    b0 = torch.randn(Cout, device=DEV) * 0.1
    dy = torch.randn(N, Cout, H, H, device=DEV)
    x, w, b = (t.clone().requires_grad_(True) for t in (x0, w0, b0))
    prev = modconv.fast_backward
    modconv.fast_backward = mode != 'composed'
    try:
        y = modconv.fused_conv(x, w, bias=b, padding=1, act='lrelu', gain=np.sqrt(2), clamp=256.0, wgain=wgain)
        grads = torch.autograd.grad((y * dy).sum(), [x, w, b], create_graph=(mode == 'create_graph'))
    finally:
        modconv.fast_backward = prev
    xr, wr, br = (t.detach().double().requires_grad_(True) for t in (x0, w0, b0))
    yr = F.leaky_relu(F.conv2d(xr, wr * wgain, br, padding=1), 0.2) * np.sqrt(2)
    ref = torch.autograd.grad((yr * dy.double()).sum(), [xr, wr, br])
    assert rel_err(y.double(), yr) < 1e-5
    for name, g, r in zip(('dx', 'dw', 'db'), grads, ref):
        assert rel_err(g.double(), r) < 1e-4, name


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(4, 256, 256), (11, 48, 256), (13, 40, 256), (3, 64, 704), (8, 256, 256)])
@pytest.mark.parametrize('form', ['mod_epi_raw', 'mod_epi', 'mod_only', 'plain_epi', 'plain', 'epi_no_noise'])
@pytest.mark.parametrize('ring', ['4', '44', '46', '49', '8', '84'])
def test_conv3x3_c64_ring(dtype, shape, form, ring, monkeypatch):
    """The 64 -> 64 channel ring kernel (LDS-DMA halo ring, weights in registers modulated per sample;
    conv3x3.hip conv3x3_c64r_kernel) in its three forms (ring 4: two workgroups per CU on 32 x 4 tiles, 2-slot rings;
    ring 44: ring 4 with whole-line stores staged through LDS; 46 (the default): ring 4 with the hoisted DMA issue;
    49: ring 46 with a per-sample dynamic tail (engaged at the (8, 256, 256) shape);
    ring 8: one workgroup of 8 waves on 32 x 8 tiles,
    3-slot ring; ring 84: the same tiles with 4 waves of 4 rows)
    and every form the layers use -- the synthesis forward
    (modulation, demod, noise, bias, lrelu, clamp, raw output), the path-length pass's scaled transposed conv
    (modulation only), the D conv (bias + lrelu + clamp), a plain conv -- against float64.  Shapes cover bands of
    4 / 2 / 1 tile rows, runs that cross samples (the per-sample weight re-modulation) and image borders on every
    side."""
    from torch_utils.ops import conv2d_gradfix as cg
    monkeypatch.setenv('SG2_C64_RING', ring)
    N, H, W = shape
    C = 64
    th = 4 if ring in ('4', '44', '46', '49') else 8
    wgs = (2 if th == 4 else 1) * torch.cuda.get_device_properties(DEV).multi_processor_count
    assert N * (H // th) * (W // 32) >= 2 * wgs      # the ring kernel's minimum of two tiles per workgroup
    torch.manual_seed(17)
    x = torch.randn(N, C, H, W)
    w = torch.randn(C, C, 3, 3) / np.sqrt(C * 9)
    s = torch.rand(N, C) + 0.5
    d = torch.rand(N, C) + 0.5
    noise = torch.randn(N, 1, H, W)
    b = torch.randn(C) * 0.1
    mod = form.startswith('mod')
    epi = 'epi' in form
    demod_noise = form.startswith('mod_epi')
    kw = {}
    if epi:
        kw.update(bias=b.to(DEV), act=1, alpha=0.2, gain=np.sqrt(2), clamp=1.5)
    if demod_noise:
        kw.update(out_scale=d.to(DEV), noise=noise.to(DEV, dtype).reshape(N, H, W).contiguous(), noise_gain=0.3)
    if form == 'epi_no_noise':
        kw.update(out_scale=d.to(DEV))
    xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv(w.to(DEV, dtype))
    y, raw = cg.conv3x3_fused(xd, wp, C, in_scale=s.to(DEV) if mod else None, want_raw=form.endswith('raw'), **kw)
    xs = (x.to(dtype).float() * s[:, :, None, None]).to(dtype).double() if mod else x.to(dtype).double()
    c = F.conv2d(xs, w.to(dtype).double(), padding=1)
    ref = c
    if epi:
        z = c * (d[:, :, None, None] if (demod_noise or form == 'epi_no_noise') else 1)
        if demod_noise:
            z = z + noise.to(dtype).double() * 0.3
        z = z + b[None, :, None, None]
        ref = (F.leaky_relu(z, 0.2) * np.sqrt(2)).clamp(-1.5, 1.5)
    tol = 5e-3 if dtype == torch.float16 else 2e-2
    assert rel_err(y.float(), ref) < tol
    if form.endswith('raw'):
        assert rel_err(raw.float(), c) < tol
    # every border pixel and every sample individually (a missed halo zero or a stale weight set shows here)
    for n in range(N):
        assert rel_err(y[n].float(), ref[n]) < 2 * tol, n
    edge = torch.zeros(H, W, dtype=torch.bool)
    edge[0], edge[-1], edge[:, 0], edge[:, -1] = True, True, True, True
    assert rel_err(y.float()[..., edge], ref[..., edge]) < 2 * tol


@pytest.mark.parametrize('form', ['mod_epi_raw', 'plain'])
def test_conv3x3_c64_ring_no_dynamic_tail(form, monkeypatch):
    """The default ring form (49) on a shape whose dynamic tail has no plan: 16 samples divide the
    2 x 256 workgroups, but each sample's 27 x 11 = 297 tiles leave an odd remainder after any even number of static
    tiles per workgroup, so the launch takes the static form 46 instead of failing."""
    test_conv3x3_c64_ring(torch.float16, (16, 108, 352), form, '49', monkeypatch)


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(4, 256, 256), (3, 344, 320), (2, 512, 256), (5, 104, 512)])
@pytest.mark.parametrize('form', ['mod_epi_raw', 'mod_epi', 'mod_only', 'plain_epi', 'plain', 'epi_no_noise'])
@pytest.mark.parametrize('ring32', ['1', '0'])
def test_conv3x3_c32_ring(dtype, shape, form, ring32, monkeypatch):
    """The 32 -> 32 channel ring kernel (conv3x3.hip conv3x3_c32r_kernel: 64-byte positions, 32 x 8 tiles, weights in
    registers modulated per sample; ring32 '0': the generic halo kernel it replaces) in every layer form against
    float64.  Shapes: bands of 4 and 1 tile rows (H / 8 = 43), runs that cross samples, every image border."""
    from torch_utils.ops import conv2d_gradfix as cg
    monkeypatch.setenv('SG2_C32_RING', ring32)
    N, H, W = shape
    C = 32
    wgs = 2 * torch.cuda.get_device_properties(DEV).multi_processor_count
    assert N * (H // 8) * (W // 32) >= 2 * wgs      # the ring kernel's minimum of two tiles per workgroup
    torch.manual_seed(19)
    x = torch.randn(N, C, H, W)
    w = torch.randn(C, C, 3, 3) / np.sqrt(C * 9)
    s = torch.rand(N, C) + 0.5
    d = torch.rand(N, C) + 0.5
    noise = torch.randn(N, 1, H, W)
    b = torch.randn(C) * 0.1
    mod = form.startswith('mod')
    epi = 'epi' in form
    demod_noise = form.startswith('mod_epi')
    kw = {}
    if epi:
        kw.update(bias=b.to(DEV), act=1, alpha=0.2, gain=np.sqrt(2), clamp=1.5)
    if demod_noise:
        kw.update(out_scale=d.to(DEV), noise=noise.to(DEV, dtype).reshape(N, H, W).contiguous(), noise_gain=0.3)
    if form == 'epi_no_noise':
        kw.update(out_scale=d.to(DEV))
    xd = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv(w.to(DEV, dtype))
    y, raw = cg.conv3x3_fused(xd, wp, C, in_scale=s.to(DEV) if mod else None, want_raw=form.endswith('raw'), **kw)
    xs = (x.to(dtype).float() * s[:, :, None, None]).to(dtype).double() if mod else x.to(dtype).double()
    c = F.conv2d(xs, w.to(dtype).double(), padding=1)
    ref = c
    if epi:
        z = c * (d[:, :, None, None] if (demod_noise or form == 'epi_no_noise') else 1)
        if demod_noise:
            z = z + noise.to(dtype).double() * 0.3
        z = z + b[None, :, None, None]
        ref = (F.leaky_relu(z, 0.2) * np.sqrt(2)).clamp(-1.5, 1.5)
    tol = 5e-3 if dtype == torch.float16 else 2e-2
    assert rel_err(y.float(), ref) < tol
    if form.endswith('raw'):
        assert rel_err(raw.float(), c) < tol
    for n in range(N):
        assert rel_err(y[n].float(), ref[n]) < 2 * tol, n
    edge = torch.zeros(H, W, dtype=torch.bool)
    edge[0], edge[-1], edge[:, 0], edge[:, -1] = True, True, True, True
    assert rel_err(y.float()[..., edge], ref[..., edge]) < 2 * tol


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize('C', [8, 64, 512])
@pytest.mark.parametrize('form', ['G_dot', 'axpy', 'act', 'scale_only'])
def test_vjp_axpy(dtype, C, form):
    """sg2_vjp_axpy (the elementwise steps of modconv._LayerVJP) against its f32 torch expression."""
    from torch_utils.ops import conv2d_gradfix as cg
    torch.manual_seed(5)
    N, H, W = 3, 17, 24
    T = lambda t: t.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    a, b, e, y = (T(torch.randn(N, C, H, W)) for _ in range(4))
    sa, sb = torch.rand(N, C, device=DEV) + 0.5, torch.randn(N, C, device=DEV)
    kw = dict(G_dot=dict(sa=sa, b=b, sb=sb, e=e), axpy=dict(b=b, sb=sb), act=dict(b=b, sb=sb, y=y),
              scale_only=dict(sa=sa))[form]
    act = dict(act=1, alpha=0.2, gain=1.41, clamp=1.0) if form == 'act' else {}
    out, dot = cg.vjp_axpy(a, **kw, **act)
    v = a.float() * (kw['sa'][:, :, None, None] if 'sa' in kw else 1)
    if 'b' in kw:
        v = v + b.float() * sb[:, :, None, None]
    if form == 'act':
        yf = y.float()
        v = torch.where(yf > 0, v, v * 0.2) * 1.41
        v = torch.where(yf.abs() < 1.0, v, torch.zeros_like(v))
    tol = {torch.float16: 1e-3, torch.bfloat16: 8e-3, torch.float32: 1e-6}[dtype]
    assert out.dtype == dtype and out.is_contiguous(memory_format=torch.channels_last)
    assert rel_err(out.float(), v) < tol
    if form == 'G_dot':
        assert rel_err(dot, (a.float() * e.float()).sum([2, 3])) < 1e-5


@pytest.mark.parametrize('up,cin,cout,res,n', [(1, 512, 512, 64, 1), (2, 512, 512, 64, 1), (1, 128, 64, 32, 3),
                                                (2, 64, 64, 64, 2), (1, 64, 64, 256, 2)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.float16])
def test_layer_vjp_matches_composed(up, cin, cout, res, n, dtype, monkeypatch):
    """The fused create_graph VJP nodes (modconv._LayerVJP, _UpLayerVJP) against the fused layer's composed VJP on
    the path-length pass (reference loss.py:85-100: the ws gradient under no_weight_gradients, then the penalty's
    backward with weight gradients on) at network widths: the f32 split-K shapes of the 64^2 / 512-channel
    blocks, the up-2 layer, and the 16-bit halo / ring layers.  Every second-order gradient (weight, bias, noise
    strength, affine, the input and the latent)."""
    from training import networks_stylegan2 as net
    from torch_utils.ops import conv2d_gradfix, modconv
    torch.manual_seed(23)
    layer = net.SynthesisLayer(cin, cout, w_dim=32, resolution=res, up=up, conv_clamp=256).to(DEV)
    with torch.no_grad():
        layer.noise_strength.fill_(0.2)
        layer.bias.copy_(torch.randn(cout) * 0.2)
    hin = res // up
    x0 = torch.randn(n, cin, hin, hin, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    w0 = torch.randn(n, 32, device=DEV)
    noise = torch.randn(n, 1, res, res, device=DEV)
    pl = torch.randn(n, cout, res, res, device=DEV) / res
    params = [layer.weight, layer.bias, layer.noise_strength, layer.affine.weight, layer.affine.bias]
    out = []
    for vjp in [True, False]:
        monkeypatch.setattr(modconv, 'fused_vjp', vjp)   # restored even if the pass raises
        x = x0.clone().requires_grad_(True)
        wv = w0.clone().requires_grad_(True)
        orig = torch.randn
        torch.randn = lambda *a, **k: noise.clone()
        try:
            y = layer(x, wv)
        finally:
            torch.randn = orig
        with conv2d_gradfix.no_weight_gradients():
            g_w, g_x = torch.autograd.grad((y.float() * pl).sum(), [wv, x], create_graph=True)
        loss = g_w.square().sum() + g_x.float().square().sum()
        g2 = torch.autograd.grad(loss, params + [x, wv], allow_unused=True)
        out.append([g_w.float(), g_x.float()] + [g if g is None else g.float() for g in g2])
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    names = ['g_w', 'g_x', 'weight', 'bias', 'noise_strength', 'affine.weight', 'affine.bias', 'x', 'wv']
    for name, a_, b_ in zip(names, *out):
        if b_ is None or float(b_.abs().max()) == 0:
            assert a_ is None or float(a_.abs().max()) == 0, name
            continue
        assert rel_err(a_, b_) < tol, (name, rel_err(a_, b_))


@pytest.mark.parametrize('geom', [(3, 1, 1, False, 2, 512, 8, 8, 512), (3, 1, 1, False, 4, 512, 4, 4, 512),
                                  (3, 1, 1, False, 4, 256, 16, 16, 128), (3, 2, 0, True, 2, 128, 9, 9, 64),
                                  (3, 2, 0, False, 3, 64, 17, 17, 48), (1, 1, 0, False, 2, 64, 16, 16, 40)])
def test_presplit_f32_accuracy(geom, monkeypatch):
    """f32 convolutions on pre-split operands (sg2_split3 + SG2_F32S3) keep f32 accuracy: forward with modulation,
    epilogue and dot (plain, split-K, strided, transposed) and the weight gradient with both scales, each within
    2e-6 of float64 and no worse than 1.5x the in-loop split's error (the two forms tile and order their sums
    differently, so they are not bitwise equal)."""
    from torch_utils.ops import conv2d_gradfix as cg
    k, stride, pad, transpose, N, Cin, H, W, Cout = geom
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, Cin, H, W, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    if transpose:
        w = (torch.randn(Cin, Cout, k, k, generator=g) / (Cin * k * k) ** 0.5).to(DEV)
        oh, ow = (H - 1) * stride - 2 * pad + k, (W - 1) * stride - 2 * pad + k
        wp = cg._pack_convT(w)
    else:
        w = (torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5).to(DEV)
        oh, ow = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
        wp = cg._pack_conv(w)
    s_in = (torch.rand(N, Cin, generator=g) + 0.5).to(DEV)
    s_out = (torch.rand(N, Cout, generator=g) + 0.5).to(DEV)
    src = torch.randn(N, Cout, oh, ow, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    gr = torch.randn(N, Cout, oh, ow, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    gs = (torch.rand(N, Cout, generator=g) + 0.5).to(DEV)
    bias = torch.randn(Cout, generator=g).to(DEV)
    out = []
    for p3 in (True, False):
        monkeypatch.setattr(cg, 'presplit', p3)
        monkeypatch.setattr(cg, 'presplit_fwd', p3)
        y, _, dot = cg.conv_fused(x, wp, Cout, oh, ow, k, k, stride, (pad, pad), transpose=transpose, in_scale=s_in,
                                  out_scale=s_out, bias=bias, act=1, gain=1.4, dot_src=src)
        res = [y, dot, cg._conv_raw(x, wp, Cout, oh, ow, k, k, stride, (pad, pad), transpose)]
        if not transpose:
            res.append(cg._wgrad_raw(gr, x, k, k, stride, (pad, pad), x_scale=s_in, g_scale=gs, alpha=0.7))
        out.append(res)
    ref = _ref_conv(x * s_in[:, :, None, None], w, stride, pad, transpose, (oh, ow))
    v = ref * s_out.double().cpu()[:, :, None, None] + bias.double().cpu()[None, :, None, None]
    refs = [torch.where(v > 0, v, 0.2 * v) * 1.4, (ref * src.double().cpu()).sum([2, 3]),
            _ref_conv(x, w, stride, pad, transpose, (oh, ow))]
    if not transpose:
        refs.append(torch.nn.grad.conv2d_weight((x * s_in[:, :, None, None]).double().cpu(), (Cout, Cin, k, k),
                                                (gr * gs[:, :, None, None]).double().cpu(), stride=stride,
                                                padding=pad) * 0.7)
    for i, r in enumerate(refs):
        e3, e = rel_err(out[0][i], r), rel_err(out[1][i], r)
        assert e3 < 2e-6 and e3 <= 1.5 * e + 1e-7, f'output {i}: pre-split err {e3:.3g}, in-loop split err {e:.3g}'


@pytest.mark.parametrize('n', [1, 37, 5000])
def test_training_stats_moments(n):
    """training_stats.report / report_sign on the device (sg2_moments, one launch) against the reference's
    moments (count, sum, sum of squares; training_stats.py:55-99) of the value and of its sign."""
    from torch_utils import training_stats as ts
    g = torch.Generator().manual_seed(n)
    v = torch.randn(n, 1, generator=g)
    v[0, 0] = 0.0
    table = ts._board.table(DEV)
    ra, rb = ts._board.row(f'test/moments/{n}'), ts._board.row(f'test/signs/{n}')
    before = table[[ra, rb]].clone()
    ts.report(f'test/moments/{n}', v.to(DEV))
    ts.report_sign(f'test/signs/{n}', v.to(DEV))
    got = (table[[ra, rb]] - before).cpu()
    vd, sd = v.double().flatten(), v.sign().double().flatten()
    want = torch.tensor([[n, vd.sum(), vd.square().sum()], [n, sd.sum(), sd.square().sum()]], dtype=torch.float64)
    assert torch.allclose(got, want, rtol=1e-12, atol=1e-9), (got, want)


@pytest.mark.gpu
def test_training_stats_sign_nan():
    """report_sign of a value holding NaN: sg2_moments' sign maps NaN to 0 as torch.sign does on the same device
    ((0 < x) - (x < 0)), so divergent logits keep Loss/signs/* finite (the ADA heuristic's input)."""
    from torch_utils import training_stats as ts
    v = torch.tensor([[1.5], [float('nan')], [-2.0], [0.0], [float('nan')]], device=DEV)
    table = ts._board.table(DEV)
    r = ts._board.row('test/signs/nan')
    before = table[r].clone()
    ts.report_sign('test/signs/nan', v)
    got = (table[r] - before).cpu()
    sd = v.sign().double().flatten().cpu()
    want = torch.tensor([v.numel(), sd.sum(), sd.square().sum()], dtype=torch.float64)
    assert torch.isfinite(got).all() and torch.equal(got, want), (got, want)


def test_vjp_nodes_upstream_gradient():
    """The path-length pass's second-order nodes with an upstream gradient that itself depends on a leaf
    (_InfNormVJP's g_dy, _DemodVJP's g_dd and g_d): the second pass differentiates into that leaf too, against
    autograd of the reference expressions (networks_stylegan2.py:52-54, :59-63) in float64."""
    from training import networks_stylegan2 as net
    from torch_utils.ops import conv2d_gradfix as cg
    torch.manual_seed(9)
    w = torch.randn(24, 20, 3, 3)
    w[3, 5, 1, 1] = w[3].abs().max() + 1.0
    w[3, 7, 0, 2] = -w[3, 5, 1, 1]
    s = torch.randn(4, 20)
    aw0, as0 = torch.randn_like(w), torch.randn_like(s)
    qw, qs = torch.randn_like(w), torch.randn_like(s)
    dd0, qd = torch.randn(4, 24), torch.randn(4, 20)

    def ref_prenorm(w_, s_):
        return (w_ * (1 / np.sqrt(20 * 9) / w_.norm(float('inf'), dim=[1, 2, 3], keepdim=True)),
                s_ / s_.norm(float('inf'), dim=1, keepdim=True))

    def ref_demod(w_, s_):
        return ((w_[None] * s_[:, None, :, None, None]).square().sum([2, 3, 4]) + 1e-8).rsqrt()

    out = []
    for dev, dt, pre, dem in [(DEV, torch.float32, net._prenorm, net._demod),
                              (torch.device('cpu'), torch.float64, ref_prenorm, ref_demod)]:
        L = lambda t: t.to(dev, dt).requires_grad_(True)  # noqa: E731
        wd, sd, aw, as_ = L(w), L(s), L(aw0), L(as0)
        yw, ys = pre(wd, sd)
        g1w, g1s = torch.autograd.grad((yw * aw).sum() + (ys * as_).sum(), [wd, sd], create_graph=True)
        r1 = torch.autograd.grad((g1w * qw.to(dev, dt)).sum() + (g1s * qs.to(dev, dt)).sum(), [wd, sd, aw, as_])
        ws, ss, ddl = L(w), L(s.abs() + 0.2), L(dd0)
        d = dem(ws, ss)
        with cg.no_weight_gradients(dev.type == 'cuda'):
            gs, = torch.autograd.grad((d * ddl).sum(), [ss], create_graph=True)
        r2 = torch.autograd.grad((gs * qd.to(dev, dt)).sum() + (d * ddl).square().sum(), [ws, ss, ddl])
        out.append([t.detach().double().cpu() for t in (*r1, *r2)])
    for i, (a, b) in enumerate(zip(*out)):
        assert rel_err(a, b) < 1e-5, (i, rel_err(a, b))
