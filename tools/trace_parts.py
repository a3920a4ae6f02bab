"""Run each part of one training iteration once, separated by idle gaps, for a rocprofv3 kernel trace:
    rocprofv3 --kernel-trace -d gpurun_out/tr -o run --output-format csv -- python tools/trace_parts.py
    python tools/trace_report.py gpurun_out/tr
Parts: synthesis fwd, D fwd, G fwd+bwd, D fwd+bwd (aug), then the loss phases Gmain, Greg, Dmain, Dreg (eager)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402


class A:
    gpus = 1; steps = 1; warmup = 0; res = 256; batch_gpu = 32; cbase = 16384; img_channels = 1; c_dim = 2
    map_depth = 8; fp16_dtype = 'fp16'; phase_timing = False


dev = torch.device('cuda', 0)
tr = bench.build(A, dev, 0, 1)
G, D, aug = tr.G, tr.D, tr.augment_pipe
z = torch.randn([32, 512], device=dev)
c = torch.nn.functional.one_hot(torch.randint(0, 2, [32], device=dev), 2).float()
with torch.no_grad():
    ws = G.mapping(z, c)
    img = G.synthesis(ws)


def part(name, fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    time.sleep(0.2)
    print('PART', name, time.clock_gettime_ns(time.CLOCK_MONOTONIC), time.clock_gettime_ns(time.CLOCK_BOOTTIME), flush=True)
    fn()
    torch.cuda.synchronize()
    time.sleep(0.2)


def syn():
    with torch.no_grad():
        G.synthesis(ws)


def dfwd():
    with torch.no_grad():
        D(img, c)


def gfb():
    G.requires_grad_(True)
    G.synthesis(G.mapping(z, c)).sum().backward()
    G.requires_grad_(False)


def dfb():
    D.requires_grad_(True)
    D(aug(img), c).sum().backward()
    D.requires_grad_(False)


real = torch.rand([32, 1, 256, 256], device=dev) * 2 - 1


def phase(name):
    # one phase's loss gradients exactly as the trainer runs them (eager; no optimizer step)
    def run():
        mod = G if name.startswith('G') else D
        mod.requires_grad_(True)
        tr.loss.accumulate_gradients(phase=name, real_img=real, real_c=c, gen_z=z, gen_c=c, gain=1, cur_nimg=0)
        mod.requires_grad_(False)
        for p in mod.parameters():
            p.grad = None
    return run


part('synthesis_fwd', syn)
part('D_fwd', dfwd)
part('G_fwd_bwd', gfb)
part('augD_fwd_bwd', dfb)
for ph in (sys.argv[1:] or ['Gmain', 'Greg', 'Dmain', 'Dreg']):
    part(ph, phase(ph))
