"""Large reductions of the training step in stages that torch never splits over workgroups.

torch reduces a tensor with few outputs and many values per output (a bias gradient: N*H*W values into each of C
outputs; a scalar noise strength's gradient: N*H*W values into one) by splitting every output over several
workgroups that meet through a staging buffer and a semaphore array, zero-filled by a memset issued with the sum.
Captured into a phase graph, that memset node is the one place where a replay differed from an identical run
(tests/test_bench_gpu.py: the 256^2 toRGB bias, 2M values into one; tools/memset_ops.py lists the sums of the bench
step that issue memsets).  Summing in stages of at most STAGE_VALUES values per output (innermost dimensions first;
two stages for every sum of the step) keeps each output inside one workgroup: no memset, a fixed order, and one
small extra launch per sum.

The reference takes these sums with torch.sum or autograd's broadcast reduction (src/models/stylegan3/torch_utils/ops/
bias_act.py:170 (db), training/networks_stylegan2.py:317-319 (noise * noise_strength)); the order of the float additions differs,
the values agree to float rounding.
"""
import torch


# Values per output of one stage.  torch splits an output over workgroups when, after spreading it over a 512-thread
# workgroup (and 4-wide vector loads), each thread would still add >= 256 values (Reduce.cuh setReduceConfig): from
# ~131K values per output upward.  65536 keeps a factor of two below that without the vector loads.
STAGE_VALUES = 65536


def staged_sum(t, dims, keepdim=False, dtype=None):
    """t.sum(dims, keepdim, dtype) in as few stages as keep every stage at <= STAGE_VALUES values per output (the
    reduced dimensions grouped innermost first: a bias gradient over [N, C, H, W] is sum([2, 3]) then sum(0));
    differentiable.  16-bit inputs are accumulated in float32 across the stages and rounded once, as torch's single
    sum does."""
    out_dtype = dtype if dtype is not None else t.dtype
    acc = torch.float32 if t.dtype in (torch.float16, torch.bfloat16) and dtype is None else dtype
    dims = sorted({d % t.ndim for d in dims}, reverse=True)
    groups, cur, vals = [], [], 1
    for d in dims:
        if cur and vals * t.shape[d] > STAGE_VALUES:
            groups.append(cur)
            cur, vals = [], 1
        cur.append(d)
        vals *= t.shape[d]
    if cur:
        groups.append(cur)
    for k, grp in enumerate(groups):
        t = t.sum(grp, keepdim=True, dtype=acc if k == 0 else None)
    if not keepdim:
        for d in dims:
            t = t.squeeze(d)
    return t.to(out_dtype)


class _ScaleByScalar(torch.autograd.Function):
    """t * s for a 0-dim parameter s with its gradient taken by staged_sum; the backward is made of differentiable
    ops (a create_graph pass differentiates through it)."""

    @staticmethod
    def forward(ctx, t, s):
        ctx.save_for_backward(t, s)
        return t * s

    @staticmethod
    def backward(ctx, g):
        t, s = ctx.saved_tensors
        gt = g * s if ctx.needs_input_grad[0] else None
        gs = staged_sum(g * t, range(g.ndim)).to(s.dtype).reshape(s.shape) if ctx.needs_input_grad[1] else None
        return gt, gs


def scale_by_scalar(t, s):
    """t * s (s a 0-dim tensor) without torch's split reduction in the gradient of s."""
    if s.ndim != 0 or not t.is_cuda:
        return t * s
    return _ScaleByScalar.apply(t, s)
