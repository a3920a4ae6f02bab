"""Timing of the ADA warp's grid-sample kernels at the 256^2 pipe's shapes (GPU): forward and input gradient, the
float-atomic scatter and the deterministic gather.  Usage: python tools/gs_micro.py"""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import sg2hip  # noqa: E402
from torch_utils.ops import grid_sample_gradfix as gs  # noqa: E402

dev = torch.device('cuda', 0)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


N, Hs, dyn, Ho = 32, 1532, 672, 560
x = torch.randn([N, 1, Hs, Hs], device=dev).requires_grad_(True)
dyn_hw = torch.tensor([dyn, dyn], dtype=torch.int32, device=dev)
g = torch.Generator(device='cpu').manual_seed(0)
ang = (torch.rand(N, generator=g) - 0.5) * 0.1
sc = 1 + (torch.rand(N, generator=g) - 0.5) * 0.1
theta = torch.zeros(N, 2, 3)
theta[:, 0, 0] = sc * torch.cos(ang)
theta[:, 0, 1] = -sc * torch.sin(ang)
theta[:, 1, 0] = sc * torch.sin(ang)
theta[:, 1, 1] = sc * torch.cos(ang)
theta = theta.to(dev)
gy = torch.randn([N, 1, Ho, Ho], device=dev)
fwd = lambda: gs.affine_grid_sample(x, theta, [N, 1, Ho, Ho], dyn_hw=dyn_hw)  # noqa: E731
print(f'fwd {timeit(lambda: fwd().detach()) * 1e3:.1f} us', flush=True)
for det in (False, True):
    with sg2hip.deterministic(det):
        t = timeit(lambda: torch.autograd.grad(fwd(), [x], gy))
    print(f'fwd + bwd det={det}: {t * 1e3:.1f} us', flush=True)
