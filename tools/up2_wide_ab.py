"""A/B of the up-2 transposed conv's 8-wave 16 x 16-cell form against the 4-wave 16 x 8 form (SG2_UP2_WIDE) on
the up / D-dgrad shapes of the bench networks (GPU): time per launch, alternating, best of three, and the two
outputs compared bitwise.    python tools/up2_wide_ab.py
(The wide form measured mixed, profiles/r06bd/, and was removed with its switch: in today's tree both legs run
the 4-wave form.)"""
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


for (n, cin, h, cout, mod) in [(32, 512, 32, 256, True), (32, 256, 64, 128, True), (32, 128, 128, 64, True),
                               (32, 512, 16, 512, True), (64, 512, 32, 256, False), (64, 256, 64, 128, False),
                               (64, 128, 128, 64, False), (16, 512, 32, 256, True)]:
    x = torch.randn(n, cin, h, h, device=dev).half().contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv((torch.randn(cout, cin, 3, 3, device=dev) / np.sqrt(cin * 9)).half())
    s = (torch.rand(n, cin, device=dev) + 0.5) if mod else None
    flops = 2.0 * n * h * h * cin * cout * 9
    t = {'1': [], '0': []}
    ys = {}
    for rep in range(3):
        for wide in ('1', '0'):
            os.environ['SG2_UP2_WIDE'] = wide
            t[wide].append(timeit(lambda: cg._conv_up2(x, wp, cout, in_scale=s)))
            ys[wide] = cg._conv_up2(x, wp, cout, in_scale=s)
    os.environ['SG2_UP2_WIDE'] = '1'
    a, b = min(t['1']), min(t['0'])
    print(f'N={n} Cin={cin} {h}^2 -> {2 * h + 1}^2 Cout={cout} mod={mod}: wide {a:.4f} ms ({flops / a / 1e9:.0f} TF) | '
          f'4-wave {b:.4f} ms ({flops / b / 1e9:.0f} TF) | x{b / a:.3f} | bitwise equal {torch.equal(ys["0"], ys["1"])}',
          flush=True)
