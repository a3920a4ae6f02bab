"""Device time of torch's own kernels in one training step, by the aten op (and input shapes) that launched them
(GPU diagnostic; eager, every phase): where the 'torch elementwise / reduce / copy' family of the step breakdown
goes, in microseconds rather than launch counts (tools/glue_census.py counts ops).
    python tools/glue_time.py [steps]"""
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
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    args = argparse.Namespace(res=256, batch_gpu=32, cbase=16384, img_channels=1, c_dim=2, map_depth=8,
                              fp16_dtype='fp16', phase_timing=False, deterministic='on')
    tr = bench.build(args, DEV, 0, 1)
    real, real_c = bench.make_inputs(args, DEV, 0)
    for _ in range(2):
        bench.one_step(tr, args, DEV, real, real_c)
    tr.batch_idx = 0
    torch.cuda.synchronize(DEV)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(steps):
            bench.one_step(tr, args, DEV, real, real_c)
        torch.cuda.synchronize(DEV)
    by_op = collections.defaultdict(lambda: [0, 0.0])
    for e in prof.events():
        for k in getattr(e, 'kernels', []):
            if 'at::native' not in k.name and 'Cijk' not in k.name:
                continue
            key = (e.name, str(e.input_shapes)[:90])
            by_op[key][0] += 1
            by_op[key][1] += k.duration
    tot = sum(v[1] for v in by_op.values()) / steps
    print(f'torch kernels: {sum(v[0] for v in by_op.values()) / steps:.0f} launches, {tot / 1e3:.3f} ms per step '
          f'(the steps here include every phase: batch_idx 0 first)', flush=True)
    for (op, shp), (n, t) in sorted(by_op.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f'{t / steps:8.1f} us/step {n / steps:6.1f}/step  {op[:34]:34s} {shp}', flush=True)


if __name__ == '__main__':
    main()
