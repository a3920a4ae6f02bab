"""A/B of the f4 FIR kernel's XCD-contiguous block order (SG2_FIR_XCD=1 default vs 0) on the D down-2 FIRs and the
narrow pad-FIRs (GPU).  Usage: python tools/fir_xcd_ab.py"""
import os, sys, torch
sys.path[:0] = ['/root/repo/gan-track_amd', '/root/repo']
from torch_utils.ops import upfirdn2d
dev = torch.device('cuda', 0)
f = upfirdn2d.setup_filter([1, 3, 3, 1], device=dev)
def timeit(fn, reps=30):
    for _ in range(3): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / reps
for dt in (torch.float16, torch.float32):
    for n, res, C in [(64, 256, 64), (64, 128, 128), (64, 64, 256), (32, 129, 128), (32, 65, 256)]:
        x = torch.randn(n, C, res, res, device=dev, dtype=dt).contiguous(memory_format=torch.channels_last)
        if res % 2 == 0:
            fn = lambda: upfirdn2d.upfirdn2d(x, f, down=2, padding=1); kind = 'down2'
            ob = x.numel() // 4
        else:
            fn = lambda: upfirdn2d.upfirdn2d(x, f, padding=1); kind = 'pad-fir'
            ob = n * C * (res - 1) ** 2
        out = {}
        for m in ('1', '0'):
            os.environ['SG2_FIR_XCD'] = m
            out[m] = (timeit(fn), fn())
        gb = (x.numel() + ob) * x.element_size() / 1e9
        print(f'{kind} {str(dt)[6:]} N={n} {res}^2 C={C}: xcd {out["1"][0]:.4f} ms ({gb / out["1"][0] * 1e3:.0f} GB/s) | '
              f'plain {out["0"][0]:.4f} ms ({gb / out["0"][0] * 1e3:.0f} GB/s) | equal {torch.equal(out["1"][1], out["0"][1])}', flush=True)
