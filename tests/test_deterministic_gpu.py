"""Deterministic mode (sg2hip.deterministic / sg2_set_deterministic): every kernel that reduces with float atomics
on the fast path -- split-K partial sums, weight-gradient pixel splits, per-(n, c) dot / bias / demodulation
reductions, the grid-sample input-gradient scatter -- is run twice in deterministic mode and must give bitwise
equal results, and must agree with the fast (atomic) path to the rounding of a different summation order.
Then one whole phase-isolated iteration at configuration width (C2) in f32 and fp16: every gradient summary and
statistic bitwise equal between two runs."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import sg2hip
from golden_util import rel_err

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)
CL = torch.channels_last


def _nhwc(t, dtype):
    return t.to(DEV).to(dtype).contiguous(memory_format=CL)


def _check(fn, tol):
    """fn() -> list of tensors.  Deterministic twice: bitwise equal; vs the atomic path: within tol (f32
    outputs), or within 1e-3 for 16-bit outputs: a sum that lands next to a rounding boundary of the 16-bit
    result rounds to the neighbouring value (one ulp, 2^-11 / 2^-8 relative) when its order changes."""
    with sg2hip.deterministic():
        a = [t.detach().clone() for t in fn()]
        b = [t.detach().clone() for t in fn()]
    ref = [t.detach().clone() for t in fn()]
    torch.cuda.synchronize()
    for i, (x, y, r) in enumerate(zip(a, b, ref)):
        assert torch.equal(x, y), f'output {i}: deterministic runs differ (max {float((x.float() - y.float()).abs().max()):.3g})'
        t = tol if x.dtype == torch.float32 else max(tol, 1e-3)
        e = rel_err(x.float(), r.double().cpu())
        assert e < t, f'output {i}: deterministic vs atomic path {e:.3g} (tol {t:g})'


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize('shape', [(2, 16, 24, 8), (3, 64, 7, 512), (4, 64, 64, 64)])
def test_det_layer_bwd(dtype, shape):
    from torch_utils.ops import conv2d_gradfix as cg
    N, H, W, C = shape
    g = torch.Generator().manual_seed(3)
    y, c, dy = (_nhwc(torch.randn(N, C, H, W, generator=g) * 2, dtype) for _ in range(3))
    d = (torch.rand(N, C, generator=g) + 0.5).to(DEV)
    _check(lambda: cg.layer_bwd(dy, y, c, d, act=1, alpha=0.2, gain=1.5, clamp=2.5), 1e-5)


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(2, 64, 20, 33, 96), (9, 64, 128, 256, 64), (2, 512, 16, 16, 512)])
def test_det_conv3x3_dot_and_wgrad(dtype, shape):
    """16-bit 3x3: the dot epilogue (generic halo kernel: per-tile slots; the persistent C = 64 shape, 9 samples
    over 256 workgroups so runs cross samples: per-(sample, workgroup, wave) slots) and the LDS-DMA weight
    gradient, plain and scaled."""
    from torch_utils.ops import conv2d_gradfix as cg
    N, Cin, H, W, Cout = shape
    g = torch.Generator().manual_seed(4)
    x = _nhwc(torch.randn(N, Cin, H, W, generator=g), dtype)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / np.sqrt(Cin * 9)).to(DEV).to(dtype)
    src = _nhwc(torch.randn(N, Cout, H, W, generator=g), dtype)
    s = (torch.rand(N, Cout, generator=g) + 0.5).to(DEV)
    gr = _nhwc(torch.randn(N, Cout, H, W, generator=g), dtype)
    xs = (torch.rand(N, Cin, generator=g) + 0.5).to(DEV)

    def fn():
        y, raw, dot = cg.conv3x3_fused(x, cg._pack_conv(w), Cout, out_scale=s, dot_src=src)
        return [y, dot, cg._wgrad_raw(gr, x, 3, 3, 1, (1, 1)), cg._wgrad_raw(gr, x, 3, 3, 1, (1, 1), x_scale=xs)]
    _check(fn, 1e-5)


@pytest.mark.parametrize('dtype', [torch.float32, torch.float16])
@pytest.mark.parametrize('geom', [(3, 1, 1, False, 2, 512, 8, 8, 512), (3, 1, 1, False, 2, 512, 4, 4, 512),
                                  (3, 2, 0, True, 2, 128, 9, 9, 64), (3, 2, 0, False, 3, 32, 12, 10, 48),
                                  (1, 1, 0, True, 3, 128, 9, 7, 3)])
def test_det_conv_fused_split_k_and_dot(dtype, geom):
    """Implicit-GEMM conv: split-K (the f32 low-resolution 512-channel layers), strided / transposed phases,
    the per-element dot epilogue, the 1x1 small-depth dot kernel; and the generic weight gradient (f32 split
    form, pixel-split slots)."""
    from torch_utils.ops import conv2d_gradfix as cg
    k, stride, pad, transpose, N, Cin, H, W, Cout = geom
    g = torch.Generator().manual_seed(29)
    x = _nhwc(torch.randn(N, Cin, H, W, generator=g), dtype)
    if transpose:
        w = (torch.randn(Cin, Cout, k, k, generator=g) / (Cin * k * k) ** 0.5).to(DEV).to(dtype)
        oh, ow = (H - 1) * stride - 2 * pad + k, (W - 1) * stride - 2 * pad + k
        wp = cg._pack_convT(w)
    else:
        w = (torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5).to(DEV).to(dtype)
        oh, ow = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
        wp = cg._pack_conv(w)
    s = (torch.rand(N, Cout, generator=g) + 0.5).to(DEV)
    src = _nhwc(torch.randn(N, Cout, oh, ow, generator=g), dtype)
    gr = _nhwc(torch.randn(N, Cout, oh, ow, generator=g), dtype)

    def fn():
        y, _, dot = cg.conv_fused(x, wp, Cout, oh, ow, k, k, stride, (pad, pad), transpose=transpose, out_scale=s,
                                  dot_src=src)
        out = [y, dot]
        if not transpose:
            out.append(cg._wgrad_raw(gr, x, k, k, stride, (pad, pad)))
        return out
    _check(fn, 1e-5)


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('cin,cout', [(1, 64), (3, 16), (64, 1), (128, 3)])
def test_det_wgrad_1x1_small_depth(dtype, cin, cout):
    from torch_utils.ops import conv2d_gradfix as cg
    g = torch.Generator().manual_seed(11)
    n, h, w = 2, 33, 47
    x = _nhwc(torch.randn(n, cin, h, w, generator=g), dtype)
    gr = _nhwc(torch.randn(n, cout, h, w, generator=g), dtype)
    gs, xs = (torch.rand(n, cout, generator=g) + 0.5).to(DEV), (torch.rand(n, cin, generator=g) + 0.5).to(DEV)
    _check(lambda: [cg._wgrad_raw(gr, x, 1, 1, 1, (0, 0), x_scale=xs, g_scale=gs)], 1e-5)


@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('case', ['s2', 's2_scaled', 'reg16_scaled'])
def test_det_wgrad_halo_phases(dtype, case):
    """Halo weight gradients: the stride-2 one-launch kernel, and the register-staged per-phase kernel (a scaled
    16^2 layer whose workgroups span several samples): slots summed in order."""
    from torch_utils.ops import conv2d_gradfix as cg
    g = torch.Generator().manual_seed(31)
    if case.startswith('s2'):
        N, Ci, Co = 3, 64, 72
        x = _nhwc(torch.randn(N, Ci, 67, 65, generator=g), dtype)
        gr = _nhwc(torch.randn(N, Co, 33, 32, generator=g), dtype)
        xs = (torch.rand(N, Ci, generator=g) + 0.5).to(DEV) if case == 's2_scaled' else None
        _check(lambda: [cg._wgrad_raw(gr, x, 3, 3, 2, (0, 0), x_scale=xs)], 1e-5)
    else:
        N, Ci, Co = 8, 128, 128
        x = _nhwc(torch.randn(N, Ci, 16, 16, generator=g), dtype)
        gr = _nhwc(torch.randn(N, Co, 16, 16, generator=g), dtype)
        xs = (torch.rand(N, Ci, generator=g) + 0.5).to(DEV)
        gs = (torch.rand(N, Co, generator=g) + 0.5).to(DEV)
        _check(lambda: [cg._wgrad_raw(gr, x, 3, 3, 1, (1, 1), x_scale=xs, g_scale=gs)], 1e-5)


def test_det_affine_grid_sample_bwd():
    """The ADA warp's input gradient: a fixed-order gather per input pixel in deterministic mode (bitwise equal
    twice), against affine_grid + grid_sample's input gradient in float64 as the atomic scatter is held
    (test_ops_gpu.py::test_affine_grid_sample), with a static buffer and a dynamic logical extent as the augment
    pipe uses it."""
    from torch_utils.ops import grid_sample_gradfix as gs
    g = torch.Generator().manual_seed(4)
    x = torch.randn(3, 3, 140, 136, generator=g)
    theta = torch.tensor([[[1.05, 0.1, 0.03], [-0.08, 0.95, -0.02]], [[0.9, -0.2, 0.1], [0.15, 1.1, 0.05]],
                          [[0.7, 0.0, -0.2], [0.0, 1.3, 0.1]]])
    size = [3, 3, 150, 146]
    dy = torch.randn(size, generator=g)
    grid = F.affine_grid(theta.double(), size, align_corners=False)
    xd = x.to(DEV).requires_grad_(True)
    refs = []
    for hw in (None, (130, 128)):
        xr = (x if hw is None else x[:, :, :hw[0], :hw[1]]).double().requires_grad_(True)
        gr, = torch.autograd.grad(F.grid_sample(xr, grid, align_corners=False), [xr], dy.double())
        refs.append(gr if hw is None else F.pad(gr, [0, 136 - hw[1], 0, 140 - hw[0]]))

    def fn():
        out = []
        for hw in (None, (130, 128)):
            dyn = None if hw is None else torch.tensor(hw, dtype=torch.int32, device=DEV)
            y = gs.affine_grid_sample(xd, theta.to(DEV), size, dyn_hw=dyn)
            gx, = torch.autograd.grad(y, [xd], dy.to(DEV))
            out.append(gx if hw is None else gx[:, :, :hw[0], :hw[1]])
        return out
    with sg2hip.deterministic():
        a = [t.clone() for t in fn()]
        b = [t.clone() for t in fn()]
    fast = fn()
    for i, (u, v, w, r) in enumerate(zip(a, b, fast, refs)):
        r = r if i == 0 else r[:, :, :130, :128]
        assert torch.equal(u, v), f'extent {i}: deterministic runs differ'
        assert rel_err(u, r) < 1e-5 and rel_err(w, r) < 1e-5, (rel_err(u, r), rel_err(w, r))


@pytest.mark.parametrize('seed', [0, 1])
def test_det_gather_matches_scatter_ada_maps(seed, monkeypatch):
    """The gather's scan box (the exact preimage widened by 1/64 output pixel) misses no contribution: bitwise equal
    to the gather scanning one pixel beyond the rounded-out box (SG2_GATHER_WIDE=1: the same candidates in the same
    order plus ones that contribute nothing), and, like the atomic scatter, equal to grid_sample's float64 gradient to the rounding of the float sampling coordinates
(2^-11 of the sum of the terms' magnitudes plus the largest |dy|), over maps drawn as the ADA pipe draws them
    (scale 2^(0.2 N(0,1)), anisotropy, rotation, translation) plus a zoom-in to a quarter and a zoom-out by 3, at
    the pipe's 2x-upsampled sizes in a static buffer with a dynamic extent."""
    from torch_utils.ops import grid_sample_gradfix as gs
    g = torch.Generator().manual_seed(100 + seed)
    n = 12
    s = torch.exp2(0.2 * torch.randn(n, generator=g))
    s[:3] = torch.tensor([0.25, 0.4, 3.0])
    a = torch.exp2(0.2 * torch.randn(n, generator=g))
    r = (torch.rand(n, generator=g) - 0.5) * 0.6
    tx, ty = torch.randn(n, generator=g) * 0.1, torch.randn(n, generator=g) * 0.1
    c, si = torch.cos(r), torch.sin(r)
    theta = torch.stack([torch.stack([s * a * c, -s * si, tx], 1), torch.stack([s * si, s / a * c, ty], 1)], 1)
    x = torch.randn(n, 1, 524, 530, generator=g)
    size = [n, 1, 512, 520]
    dy = torch.randn(size, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    dyn = torch.tensor([500, 516], dtype=torch.int32, device=DEV)

    def fn():
        y = gs.affine_grid_sample(xd, theta.float().to(DEV), size, dyn_hw=dyn)
        return torch.autograd.grad(y, [xd], dy.to(DEV))[0][:, :, :500, :516]
    with sg2hip.deterministic():
        u = fn().clone()
        monkeypatch.setenv('SG2_GATHER_WIDE', '1')
        wide = fn().clone()
        monkeypatch.delenv('SG2_GATHER_WIDE')
    assert torch.equal(u, wide), f'{int((u != wide).sum())} pixels differ from the wide scan'
    w = fn()
    xr = x[:, :, :500, :516].double().requires_grad_(True)
    grid = F.affine_grid(theta.double(), size, align_corners=False)
    ref, = torch.autograd.grad(F.grid_sample(xr, grid, align_corners=False), [xr], dy.double())
    mag, = torch.autograd.grad(F.grid_sample(xr, grid, align_corners=False), [xr], dy.double().abs())
    # the float sampling coordinates (|ix| up to ~10^3, a few roundings of 2^-24) move each bilinear weight by up to
    # ~2^-12 (and, at a pixel boundary, a weight that small to the neighbouring pixel): a missed contribution of
    # weight >= 2^-9 is caught
    tol = 2.0 ** -11 * (mag + float(dy.abs().max()))
    for name, got in (('gather', u), ('scatter', w)):
        err = (got.double().cpu() - ref).abs()
        bad = err > tol
        assert not bool(bad.any()), (f'{name}: {int(bad.sum())} pixels off the float64 gradient, max '
                                     f'{float(err.max()):.3g}, in samples {sorted(set(bad.nonzero()[:, 0].tolist()))}')


def test_det_dot_hw_and_vjp_axpy():
    from torch_utils.ops import conv2d_gradfix as cg
    g = torch.Generator().manual_seed(5)
    a = _nhwc(torch.randn(3, 64, 37, 41, generator=g), torch.float16)
    b = _nhwc(torch.randn(3, 64, 37, 41, generator=g), torch.float16)
    _check(lambda: [cg.dot_hw(a, b)], 1e-5)


@pytest.mark.timeout(300)
@pytest.mark.parametrize('dt', [None, 'fp16'])
def test_det_isolated_iteration_c2(dt):
    """A whole phase-isolated iteration at the C2 configuration's width (256^2, cbase 16384, batch 4), twice in
    deterministic mode: every gradient summary (norm and sampled entries), pl_mean and every reported statistic
    bitwise equal."""
    import config_parity as cp
    from golden_util import load
    fdt = None if dt is None else torch.float16
    runs = []
    for _ in range(2):
        cfg, inp, tape, fix = cp.load_fixture(load('train_c2_iso.npz'))
        runs.append(cp.run_product(cfg, inp, tape, DEV, fp16_dtype=fdt, isolated=True, deterministic=True))
    (g1, s1), (g2, s2) = runs
    assert sorted(g1) == sorted(g2)
    diff = [k for k in g1 if not np.array_equal(np.asarray(g1[k]), np.asarray(g2[k]))]
    assert not diff, f'{len(diff)} summaries differ between deterministic runs, e.g. {diff[:3]}'
    for (n1, v1), (n2, v2) in zip(s1, s2):
        assert n1 == n2 and np.array_equal(v1, v2), n1


def test_det_affine_grid_sample_bwd_singular():
    """A singular affine map (det 0: both output axes sample along one input line): the deterministic gather has
    no finite inverse to bound its scan, so it scans the whole output; its input gradient must still equal
    grid_sample's in float64, as the atomic scatter's does."""
    from torch_utils.ops import grid_sample_gradfix as gs
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, 3, 40, 36, generator=g)
    theta = torch.tensor([[[0.5, 0.5, 0.1], [0.5, 0.5, -0.1]], [[0.0, 0.0, 0.2], [0.0, 0.0, 0.3]]])
    size = [2, 3, 44, 40]
    dy = torch.randn(size, generator=g)
    grid = F.affine_grid(theta.double(), size, align_corners=False)
    xr = x.double().requires_grad_(True)
    ref, = torch.autograd.grad(F.grid_sample(xr, grid, align_corners=False), [xr], dy.double())
    xd = x.to(DEV).requires_grad_(True)

    def fn():
        y = gs.affine_grid_sample(xd, theta.to(DEV), size)
        return torch.autograd.grad(y, [xd], dy.to(DEV))[0]
    with sg2hip.deterministic():
        u = fn().clone()
    w = fn()
    assert rel_err(u, ref) < 1e-5 and rel_err(w, ref) < 1e-5, (rel_err(u, ref), rel_err(w, ref))


@pytest.mark.parametrize('geom', [(512, 512, 3, 1, 1, 2, 8, 8), (64, 40, 3, 1, 1, 3, 10, 9), (40, 104, 3, 2, 0, 2, 17, 17),
                                  (48, 136, 1, 1, 0, 2, 12, 12), (8, 520, 3, 1, 1, 1, 4, 4)])
@pytest.mark.parametrize('layout', [True, 'swap'])
def test_det_wgrad_param_layout(geom, layout):
    """The f32 weight gradient's fixed-order slot sum written straight into the parameter layout
    (sg2_conv2d_wgrad_oikk: [A, B, kh, kw], or [B, A, kh, kw] for 'swap'; an LDS-transposed tile of one a x 64 b per
    workgroup): contiguous in that layout, deterministic, equal to the K-major slot sum's permuted view to the
    rounding of its summation order, and to a float64
    weight gradient; B not a multiple of 64, 1x1 and stride-2 forms included."""
    from torch_utils.ops import conv2d_gradfix as cg
    A, B, k, stride, pad, N, H, W = geom
    g = torch.Generator().manual_seed(41)
    x = _nhwc(torch.randn(N, B, H, W, generator=g), torch.float32)
    oh, ow = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    gr = _nhwc(torch.randn(N, A, oh, ow, generator=g), torch.float32)
    with sg2hip.deterministic():
        p1 = cg._wgrad_raw(gr, x, k, k, stride, (pad, pad), alpha=0.5, param_layout=layout).clone()
        p2 = cg._wgrad_raw(gr, x, k, k, stride, (pad, pad), alpha=0.5, param_layout=layout)
        plain = cg._wgrad_raw(gr, x, k, k, stride, (pad, pad), alpha=0.5)
        torch.cuda.synchronize()
    assert p2.shape == (A, B, k, k)
    assert (p2.transpose(0, 1) if layout == 'swap' else p2).is_contiguous()
    assert torch.equal(p1, p2), 'parameter-layout weight gradient not deterministic'
    ref = 0.5 * torch.nn.grad.conv2d_weight(x.double().cpu(), (A, B, k, k), gr.double().cpu(), stride=stride,
                                            padding=pad)
    e_plain = rel_err(p2, plain.double().cpu())
    assert e_plain < 1e-6, f'parameter layout vs K-major slot sum {e_plain:.3g}'
    e_ref = rel_err(p2, ref)
    assert e_ref < 1e-5, f'parameter layout vs float64 {e_ref:.3g}'
