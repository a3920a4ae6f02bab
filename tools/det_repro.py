"""Run-to-run reproducibility of the bench step (GPU diagnostic): two fresh runs of bench.build + one_step with the
same seeds, snapshots of every G / D parameter after each step; prints per step how many tensors differ and the
first ones (in registration order), for eager steps and for phase-graph replays.
    python tools/det_repro.py [steps] [graphs 0|1] [deterministic on|off]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402

DEV = torch.device('cuda', 0)


def run(steps, graphs, det):
    args = argparse.Namespace(res=256, batch_gpu=32, cbase=16384, img_channels=1, c_dim=2, map_depth=8,
                              fp16_dtype='fp16', phase_timing=False, deterministic=det)
    tr = bench.build(args, DEV, 0, 1)
    real, real_c = bench.make_inputs(args, DEV, 0)
    snaps = []
    grads = {}

    def on_grads(name, module):
        grads.setdefault(name, {k: p.grad.detach().clone() for k, p in module.named_parameters() if p.grad is not None})
    if not graphs:
        tr.on_grads = on_grads
    for s in range(steps):
        if graphs and s == 1:
            tr.graphs = True
            tr.batch_idx = 0
        bench.one_step(tr, args, DEV, real, real_c)
        torch.cuda.synchronize(DEV)
        snaps.append({f'{n}.{k}': v.detach().clone() for n, m in (('G', tr.G), ('D', tr.D))
                      for k, v in m.named_parameters()})
    return snaps, grads


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    graphs = (sys.argv[2] if len(sys.argv) > 2 else '0') == '1'
    det = sys.argv[3] if len(sys.argv) > 3 else 'on'
    a, ga = run(steps, graphs, det)
    b, gb = run(steps, graphs, det)
    for ph in ga:
        d = [k for k in ga[ph] if not torch.equal(ga[ph][k], gb[ph][k])]
        print(f'first-step {ph} gradients: {len(d)} of {len(ga[ph])} differ: {d[:6]}', flush=True)
    for s in range(steps):
        d = [k for k in a[s] if not torch.equal(a[s][k], b[s][k])]
        print(f'graphs={graphs} det={det} step {s}: {len(d)} of {len(a[s])} parameters differ: {d[:6]}', flush=True)


if __name__ == '__main__':
    main()
