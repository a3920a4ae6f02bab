"""A/B of the up-2 transposed conv's workgroup order (SG2_UP2_ORDER: 0 channel-block major, 1 XCD-contiguous
tile-major) on the up / D-dgrad shapes of the bench networks (GPU): time per launch, alternating, and the two
outputs compared bitwise (the order changes which workgroup computes a tile, not the arithmetic).
    python tools/up2_order_ab.py
(The XCD order measured slower, profiles/r06ay/, and was removed with its switch: in today's tree both legs run
the block-major order.)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

dev = torch.device('cuda', 0)


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


for (n, cin, h, cout) in [(32, 512, 32, 256), (32, 256, 64, 128), (32, 128, 128, 64), (32, 512, 16, 512),
                          (64, 512, 32, 256), (64, 256, 64, 128), (64, 128, 128, 64), (16, 512, 32, 256)]:
    x = torch.randn(n, cin, h, h, device=dev).half().contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv((torch.randn(cout, cin, 3, 3, device=dev) / np.sqrt(cin * 9)).half())
    flops = 2.0 * n * h * h * cin * cout * 9
    t = {0: [], 1: []}
    ys = {}
    for rep in range(3):
        for order in (1, 0):
            os.environ['SG2_UP2_ORDER'] = str(order)
            t[order].append(timeit(lambda: cg._conv_up2(x, wp, cout)))
            ys[order] = cg._conv_up2(x, wp, cout)
    os.environ['SG2_UP2_ORDER'] = '1'
    a, b = min(t[1]), min(t[0])
    print(f'N={n} Cin={cin} {h}^2 -> {2 * h + 1}^2 Cout={cout}: XCD order {a:.4f} ms ({flops / a / 1e9:.0f} TF) | '
          f'block-major {b:.4f} ms ({flops / b / 1e9:.0f} TF) | bitwise equal {torch.equal(ys[0], ys[1])}', flush=True)
