"""layer_bwd timing on the 256^2 network's layer shapes (GPU): bytes moved / time.
Usage: python tools/lb_micro.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402
import sg2hip  # noqa: E402

dev = torch.device('cuda', 0)
CL = torch.channels_last


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


for (n, c, h) in [(32, 64, 256), (32, 128, 128), (32, 256, 64), (32, 512, 32)]:
    mk = lambda: torch.randn(n, c, h, h, device=dev).half().contiguous(memory_format=CL)
    dy, y, cc = mk(), mk(), mk()
    d = torch.rand(n, c, device=dev) + 0.5
    for with_c in (True, False):
        for det in (False, True):
            fn = lambda: cg.layer_bwd(dy, y, cc if with_c else None, d, act=1, gain=1.41, clamp=256.0,
                                      want_db=True, want_dd=with_c, want_dnoise=with_c)
            with sg2hip.deterministic(det):
                t = timeit(fn)
            nbytes = dy.numel() * 2 * (4 if with_c else 3)
            print(f'form={os.environ.get("SG2_LB_FORM", "0")} N={n} C={c} {h}^2 c={with_c} det={det}: {t * 1e3:.1f} us, '
                  f'{nbytes / t / 1e9:.2f} TB/s', flush=True)
