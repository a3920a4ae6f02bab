"""The timed step itself, at BASELINE's full single-GPU size (bench.py: 256^2 1-ch, cbase 16384, map 8, c_dim 2, batch
32, ADA p = 0.2, fp16 top blocks), through bench.build / bench.one_step exactly as the bench runs it -- eager
warm-up, phase-graph capture, graph replays: the iteration's default arithmetic (the deterministic reductions,
Trainer(deterministic=True)) makes the whole step a function of the seeds, so two fresh runs end bitwise equal on
every parameter of G, D and G_ema and on the ADA probability.  A size-independent property of the bench
configuration, which no CPU evaluation reaches (the phase-isolated parity at these widths: test_config_gpu.py)."""
import argparse

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


def _run(steps=4):
    import bench
    args = argparse.Namespace(res=256, batch_gpu=32, cbase=16384, img_channels=1, c_dim=2, map_depth=8,
                              fp16_dtype='fp16', phase_timing=False, deterministic='on')
    tr = bench.build(args, DEV, 0, 1)
    real, real_c = bench.make_inputs(args, DEV, 0)
    snaps = []
    for s in range(steps):
        if s == 1:                                       # step 0 eager (every lazily created state), then the
            tr.graphs = True                             # phase graphs: step 1 captures, later steps replay
            tr.batch_idx = 0
        bench.one_step(tr, args, DEV, real, real_c)
        torch.cuda.synchronize(DEV)
        snap = {f'{n}.{k}': v.detach().clone() for n, m in (('G', tr.G), ('D', tr.D), ('G_ema', tr.G_ema))
                for k, v in m.named_parameters()}
        snap['aug.p'] = tr.augment_pipe.p.detach().clone()
        snaps.append(snap)
    return snaps


@pytest.mark.timeout(400)
def test_bench_step_bitwise_reproducible():
    a = _run()
    b = _run()
    for s, (x, y) in enumerate(zip(a, b)):
        assert x.keys() == y.keys()
        diff = [k for k in x if not torch.equal(x[k], y[k])]
        assert not diff, f'step {s}: {len(diff)} of {len(x)} tensors differ between two runs, e.g. {diff[:4]}'
    nonfinite = [k for k, v in a[-1].items() if not torch.isfinite(v).all()]
    assert not nonfinite, nonfinite[:3]


@pytest.mark.timeout(300)
def test_bench_step_issues_no_memsets():
    """No op of the step issues a device memset: captured into a phase graph, torch's split-reduction memset made
    the 256^2 toRGB bias gradient differ between two identical runs (torch_utils/ops/staged_sum.py).  The library
    zeroes its accumulators with kernels (csrc zero_fill), and the large sums are staged."""
    import bench
    from torch.profiler import ProfilerActivity, profile
    args = argparse.Namespace(res=256, batch_gpu=32, cbase=16384, img_channels=1, c_dim=2, map_depth=8,
                              fp16_dtype='fp16', phase_timing=False, deterministic='on')
    tr = bench.build(args, DEV, 0, 1)
    real, real_c = bench.make_inputs(args, DEV, 0)
    bench.one_step(tr, args, DEV, real, real_c)
    tr.batch_idx = 0                                     # every phase, the regularisation passes included
    torch.cuda.synchronize(DEV)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        bench.one_step(tr, args, DEV, real, real_c)
        torch.cuda.synchronize(DEV)
    ops = [(e.name, str(e.input_shapes)[:100]) for e in prof.events() for k in getattr(e, 'kernels', [])
           if 'memset' in k.name.lower()]
    n_dev = sum(1 for e in prof.events() if e.device_type.name == 'CUDA' and 'memset' in e.name.lower())
    assert n_dev == 0 and not ops, f'{n_dev} device memsets, issued by {ops[:4]}'
