"""Which ops of the training step issue device memsets (GPU diagnostic)?

A memset issued inside a phase-graph capture becomes a memset node of the graph; torch's cross-workgroup
reductions issue one (their semaphore array) and one such sum made the toRGB bias gradient differ between two
identical graph-mode runs.  This profiles one eager step of the bench configuration and lists, per aten op and
input shapes, the memsets it issued.

    python tools/memset_ops.py
"""
import argparse
import collections
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402

DEV = torch.device('cuda', 0)


def main():
    args = argparse.Namespace(res=256, batch_gpu=32, cbase=16384, img_channels=1, c_dim=2, map_depth=8,
                              fp16_dtype='fp16', phase_timing=False, deterministic='on')
    tr = bench.build(args, DEV, 0, 1)
    real, real_c = bench.make_inputs(args, DEV, 0)
    bench.one_step(tr, args, DEV, real, real_c)
    tr.batch_idx = 0                      # every phase (Greg / Dreg included) in the profiled step
    torch.cuda.synchronize(DEV)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        bench.one_step(tr, args, DEV, real, real_c)
        torch.cuda.synchronize(DEV)
    found = collections.Counter()
    for e in prof.events():
        for k in getattr(e, 'kernels', []):
            nm = k.name.lower()
            if 'memset' in nm:
                found[(e.name, str(e.input_shapes)[:120])] += 1
    dev_memsets = sum(1 for e in prof.events() if e.device_type.name == 'CUDA' and 'memset' in e.name.lower())
    print(f'device memset events: {dev_memsets}; attributed to ops: {sum(found.values())}', flush=True)
    for (op, shapes), n in found.most_common():
        print(f'{n:5d}  {op}  {shapes}', flush=True)
    names = collections.Counter(e.name for e in prof.events() if 'memset' in e.name.lower())
    print('memset event names:', dict(names), flush=True)


if __name__ == '__main__':
    main()
