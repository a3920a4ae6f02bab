"""Time the parts of one training iteration (GPU events): mapping, synthesis fwd, synthesis fwd+bwd,
augment, D fwd, D fwd+bwd, Adam.  Usage: python tools/part_timing.py"""
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


ONLY = sys.argv[1] if len(sys.argv) > 1 else None
dev = torch.device('cuda', 0)
tr = bench.build(A, dev, 0, 1)
G, D, aug = tr.G, tr.D, tr.augment_pipe
z = torch.randn([32, 512], device=dev)
c = torch.nn.functional.one_hot(torch.randint(0, 2, [32], device=dev), 2).float()


def t(name, fn, reps=5):
    if ONLY and ONLY not in name:
        return
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h0 = time.perf_counter()
    e0.record()
    issue = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()           # empty queue: the host time of fn() is its pure issue cost
        t0 = time.perf_counter()
        fn()
        issue += time.perf_counter() - t0
    e1.record()
    e1.synchronize()
    h1 = time.perf_counter()
    print(f'{name:28s} gpu {e0.elapsed_time(e1) / reps:8.2f} ms   wall {(h1 - h0) / reps * 1e3:8.2f} ms   '
          f'host issue {issue / reps * 1e3:8.2f} ms', flush=True)


with torch.no_grad():
    ws = G.mapping(z, c)
    t('mapping fwd', lambda: G.mapping(z, c))
    t('synthesis fwd (no grad)', lambda: G.synthesis(ws))
    img = G.synthesis(ws)
    t('augment fwd (no grad)', lambda: aug(img))
    t('D fwd (no grad)', lambda: D(img, c))

G.requires_grad_(True)


def gfb():
    w_ = G.mapping(z, c)
    im = G.synthesis(w_)
    im.sum().backward()


t('G fwd+bwd (params)', gfb)
G.requires_grad_(False)
D.requires_grad_(True)


def dfb():
    im = img.detach().requires_grad_(False)
    D(aug(im), c).sum().backward()


t('aug+D fwd+bwd (params)', dfb)


def dfb_noaug():
    D(img, c).sum().backward()


t('D fwd+bwd (params, no aug)', dfb_noaug)
D.requires_grad_(False)


def gmain():
    tr.loss.accumulate_gradients('Gmain', img, c, z, c, 1, 0)


G.requires_grad_(True)
t('Gmain accumulate', gmain)
G.requires_grad_(False)
