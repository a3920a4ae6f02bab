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


def _run(steps=3):
    import bench
    args = argparse.Namespace(res=256, batch_gpu=32, cbase=16384, img_channels=1, c_dim=2, map_depth=8,
                              fp16_dtype='fp16', phase_timing=False, deterministic='on')
    tr = bench.build(args, DEV, 0, 1)
    real, real_c = bench.make_inputs(args, DEV, 0)
    bench.one_step(tr, args, DEV, real, real_c)          # eager warm-up (every lazily created state)
    tr.graphs = True
    tr.batch_idx = 0
    for _ in range(steps):                               # step 0 captures every phase, later steps replay
        bench.one_step(tr, args, DEV, real, real_c)
    torch.cuda.synchronize(DEV)
    out = {}
    for name, m in (('G', tr.G), ('D', tr.D), ('G_ema', tr.G_ema)):
        for k, v in m.state_dict().items():
            out[f'{name}.{k}'] = v.detach().clone()
    out['aug.p'] = tr.augment_pipe.p.detach().clone()
    return out


@pytest.mark.timeout(400)
def test_bench_step_bitwise_reproducible():
    a = _run()
    b = _run()
    assert a.keys() == b.keys()
    diff = [k for k in a if not torch.equal(a[k], b[k])]
    assert not diff, f'{len(diff)} of {len(a)} tensors differ between two runs of the bench step, e.g. {diff[:3]}'
    nonfinite = [k for k, v in a.items() if v.is_floating_point() and not torch.isfinite(v).all()]
    assert not nonfinite, nonfinite[:3]
