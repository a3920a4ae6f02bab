"""A/B of the up-2 4x4 NHWC FIR (GPU): upfirdn_nhwc_up2 (default, a 2 x 2 output cell per lane) vs
upfirdn_nhwc_vec (SG2_UPF_UP2_OFF=1; the r04_v4 run also timed its former 64-bit index math) on the FIRs it
serves in the step -- the adjoints of the D skips' down-2 FIR (upsample2d of the gradient,
gain 4) at 128^2 x 64 ch ... 8^2 x 512 ch, bs64 and bs32.  Bitwise equality and GB/s (input + output bytes)
are printed.  Usage: python tools/upf_vec_ab.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from torch_utils.ops import upfirdn2d as upf  # noqa: E402

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


f = upf.setup_filter([1, 3, 3, 1], device=dev)
ok, tot = True, {'0': 0.0, '1': 0.0}
for n in (64, 32):
    for (c, h) in ((64, 128), (128, 64), (256, 32), (512, 16), (512, 8)):
        x = torch.randn(n, c, h, h, device=dev).half().contiguous(memory_format=torch.channels_last)
        fn = lambda: upf.upsample2d(x, f, up=2)
        res = {}
        for mode in ('0', '1'):
            os.environ.pop('SG2_UPF_UP2_OFF', None)
            if mode == '1':
                os.environ['SG2_UPF_UP2_OFF'] = '1'
            t = timeit(fn)
            res[mode] = (t, fn())
            tot[mode] += t
        y = res['0'][1]
        same = torch.equal(y, res['1'][1])
        ok &= same
        gb = (x.numel() + y.numel()) * 2 / 1e9
        print(f'up2 N={n} C={c} {h}^2 -> {y.shape[2]}^2: cell kernel {res["0"][0]:.4f} ms ({gb / res["0"][0] * 1e3:.0f} GB/s)'
              f' | vec {res["1"][0]:.4f} ms ({gb / res["1"][0] * 1e3:.0f} GB/s) | bitwise {same}', flush=True)
print(f'total cell {tot["0"]:.3f} ms, vec {tot["1"]:.3f} ms; {"ALL BITWISE EQUAL" if ok else "MISMATCH"}')
