"""The synthesis network's grouped affine layers (training/networks_stylegan2.py grouped_styles: one GEMM for all
layers' styles) against the per-layer FullyConnectedLayer path it replaces (reference networks_stylegan2.py:111-125
and :352): styles, their first-order gradients (w, weights, biases) and the second-order gradient the path-length
pass takes through them.  Host logic (torch ops), run on CPU."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gan-track_amd'))


def _net():
    from training import networks_stylegan2 as net
    torch.manual_seed(3)
    G = net.Generator(z_dim=16, c_dim=0, w_dim=32, img_resolution=32, img_channels=1, channel_base=256,
                      channel_max=64, mapping_kwargs=dict(num_layers=2))
    for m in G.modules():            # non-trivial biases and gains
        if isinstance(m, net.FullyConnectedLayer) and m.bias is not None:
            with torch.no_grad():
                m.bias.add_(torch.randn_like(m.bias) * 0.3)
    return net, G.synthesis


def _plan(syn):
    plan, w_idx = [], 0
    for r in syn.block_resolutions:
        block = getattr(syn, f'b{r}')
        plan += [(a, w_idx + k, g) for a, k, g in block.style_layers()]
        w_idx += block.num_conv
    return plan


@pytest.mark.parametrize('n', [1, 3])
def test_grouped_styles_match_per_layer(n):
    net, syn = _net()
    plan = _plan(syn)
    assert len(plan) == 3 * len(syn.block_resolutions) - 1 and plan[-1][1] == syn.num_ws - 1
    ws = torch.randn(n, syn.num_ws, 32, requires_grad=True)
    r = [torch.randn(n, a.out_features) for a, _, _ in plan]
    params = [p for a, _, _ in plan for p in (a.weight, a.bias)]
    for p in params:
        p.requires_grad_(True)

    def run(grouped):
        st = net.grouped_styles(ws, plan) if grouped else [a(ws[:, k], out_gain=g) for a, k, g in plan]
        loss = sum((s * rr).sum() for s, rr in zip(st, r))
        gw, *gp = torch.autograd.grad(loss, [ws] + params, create_graph=True)
        pl = (gw.square().sum(2) + 1).sqrt().mean()        # a path-length-like second pass through the styles
        g2 = torch.autograd.grad(pl, [ws] + params, allow_unused=True)
        g2 = [torch.zeros_like(q) if g is None else g for g, q in zip(g2, [ws] + params)]
        return st, gw, gp, g2

    a, b = run(True), run(False)
    for x, y in zip(a[0], b[0]):
        assert x.is_contiguous() and x.shape == y.shape
        assert torch.allclose(x, y, rtol=1e-5, atol=1e-6)
    assert torch.allclose(a[1], b[1], rtol=1e-5, atol=1e-6)
    for x, y in zip(a[2], b[2]):
        assert torch.allclose(x, y, rtol=1e-5, atol=1e-5)
    for x, y in zip(a[3], b[3]):
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-6)


def test_grouped_styles_plan_follows_widths():
    """Two networks of different widths built one after the other (the first freed, so its module ids may be
    reused): each one's grouped styles equal its per-layer affine (the style plan's cache key holds the layers'
    widths and gains, not their identities)."""
    from training import networks_stylegan2 as net
    for cmax in (64, 32, 64):
        torch.manual_seed(cmax)
        G = net.Generator(z_dim=16, c_dim=0, w_dim=32, img_resolution=32, img_channels=1, channel_base=256,
                          channel_max=cmax, mapping_kwargs=dict(num_layers=2))
        for m in G.modules():
            if isinstance(m, net.FullyConnectedLayer) and m.bias is not None:
                with torch.no_grad():
                    m.bias.add_(torch.randn_like(m.bias) * 0.3)
        plan = _plan(G.synthesis)
        ws = torch.randn(2, G.synthesis.num_ws, 32)
        with torch.no_grad():
            got = net.grouped_styles(ws, plan)
            ref = [a(ws[:, k], out_gain=g) for a, k, g in plan]
        for x, y in zip(got, ref):
            assert x.shape == y.shape
            assert torch.allclose(x, y, rtol=1e-5, atol=1e-6)
        del G, plan
