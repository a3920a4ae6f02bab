"""torch_utils/ops/staged_sum.py on the host: the one-dimension-at-a-time sums equal torch.sum (to float rounding),
keep 16-bit inputs in a float32 accumulator, and the scalar-scale node's gradients (first and second order) match
autograd's broadcast reduction."""
import pytest
import torch

from torch_utils.ops import staged_sum as ss


@pytest.mark.parametrize('dims', [(0, 2, 3), (2, 3), (0,), (1,), (0, 1, 2, 3), (-1, -2)])
@pytest.mark.parametrize('keepdim', [False, True])
def test_staged_sum_matches_sum(dims, keepdim):
    t = torch.randn(4, 3, 9, 7, dtype=torch.float64)
    ref = t.sum(list(dims), keepdim=keepdim)
    got = ss.staged_sum(t, dims, keepdim=keepdim)
    assert got.shape == ref.shape
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12)


def test_staged_sum_16bit_accumulates_in_f32():
    t = torch.full([8, 1, 64, 64], 1.0, dtype=torch.float16)     # 32768 ones: an f16 accumulator stops at 2048
    assert ss.staged_sum(t, (0, 2, 3)).item() == 32768.0
    assert ss.staged_sum(t, (0, 2, 3), dtype=torch.float32).dtype == torch.float32
    assert ss.staged_sum(t, (2, 3)).dtype == torch.float16


def test_scale_by_scalar_gradients():
    x = torch.randn(2, 1, 5, 5, dtype=torch.float64, requires_grad=True)
    s = torch.tensor(0.3, dtype=torch.float64, requires_grad=True)
    f = ss._ScaleByScalar.apply
    assert torch.autograd.gradcheck(f, (x, s))
    assert torch.autograd.gradgradcheck(f, (x, s))
    g = torch.randn(2, 1, 5, 5, dtype=torch.float64)
    a = torch.autograd.grad(f(x, s), (x, s), g)
    b = torch.autograd.grad(x * s, (x, s), g)
    for u, v in zip(a, b):
        torch.testing.assert_close(u, v)
