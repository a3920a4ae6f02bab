"""A/B of the stride-2 transposed 3x3 conv: sg2_conv3x3_up2 vs the generic implicit GEMM (sg2_conv2d,
four phases) on the up layers' shapes of the 256^2 / 512^2 networks (GPU).  Usage: python tools/up2_ab.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import sg2hip as _hip  # noqa: E402
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

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


def generic(x, wp, cout):
    n, cin, h, w = x.shape
    y = torch.empty([n, cout, 2 * h + 1, 2 * w + 1], dtype=x.dtype, device=dev, memory_format=torch.channels_last)
    _hip.check(_hip.lib().sg2_conv2d(_hip.ptr(y), _hip.ptr(x), _hip.ptr(wp), _hip.dtype_code(x), n, cin, h, w, cout,
                                     2 * h + 1, 2 * w + 1, 3, 3, 2, 0, 0, 1, None, 0, _hip.stream_ptr(dev)), 'sg2_conv2d')
    return y


for (n, cin, h, cout) in [(32, 128, 128, 64), (32, 256, 64, 128), (32, 512, 32, 256), (32, 512, 16, 512),
                          (64, 256, 64, 128), (64, 512, 32, 256), (64, 512, 16, 512), (64, 512, 8, 512),
                          (16, 256, 128, 128), (8, 512, 64, 256)]:
    x = torch.randn(n, cin, h, h, device=dev).half().contiguous(memory_format=torch.channels_last)
    wp = cg._pack_conv((torch.randn(cout, cin, 3, 3, device=dev) / np.sqrt(cin * 9)).half())
    flops = 2.0 * n * h * h * cin * cout * 9
    a = timeit(lambda: cg._conv_up2(x, wp, cout))
    ys = cg._conv_up2(x, wp, cout)
    os.environ['SG2_UP2_EDGE'] = '0'              # the ragged 16 x 8 tiling of all (H+1) x (W+1) cells
    r = timeit(lambda: cg._conv_up2(x, wp, cout))
    same = torch.equal(ys, cg._conv_up2(x, wp, cout))
    os.environ['SG2_UP2_EDGE'] = '1'
    b = timeit(lambda: generic(x, wp, cout))
    err = (ys.float() - generic(x, wp, cout).float()).norm() / generic(x, wp, cout).float().norm()
    print(f'N={n} Cin={cin} {h}^2 -> {2 * h + 1}^2 Cout={cout}: up2 {a:.3f} ms ({flops / a / 1e9:.0f} TF) | ragged '
          f'{r:.3f} ms (split == ragged: {same}) | generic {b:.3f} ms ({flops / b / 1e9:.0f} TF) | rel diff {err:.1e}',
          flush=True)
