"""Times the 256^2 C=64 fused synthesis-layer launch (bench.py's roofline launch) in this process's kernel
configuration (SG2_C64_RING, SG2_RING_DBG); prints ms per launch and the fraction of 8 TB/s.  Also the DOT (dgrad)
and plain forms.  Usage: python tools/ring_ab.py [reps]"""
import os
import sys
import time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

dev = torch.device('cuda', 0)
# warm the clocks first (the first launches of a cold process run ~10 % slower than the bench's, which follow
# the training steps)
_t0 = time.time()
while time.time() - _t0 < 1.0:
    bench._layer_launch(dev, 256, 64, torch.float16)
torch.cuda.synchronize()
res = []
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    ms, fl, by = bench._layer_launch(dev, 256, 64, torch.float16)
    res.append(ms)
print(f"ring={os.environ.get('SG2_C64_RING', '49')} dbg={os.environ.get('SG2_RING_DBG', '0')} fused launch ms "
      f"{' '.join(f'{m:.4f}' for m in res)}  best frac {by / (min(res) * 1e-3) / 8e12:.3f}", flush=True)
# plain conv (D layer form: bias + lrelu, no modulation) and the dgrad DOT form
N, C, R = 32, 64, 256
x = torch.randn([N, C, R, R], device=dev, dtype=torch.float16).contiguous(memory_format=torch.channels_last)
wp = cg._pack_conv((torch.randn([C, C, 3, 3], device=dev) / 24).to(torch.float16))
b = torch.zeros([C], device=dev)
s = torch.rand([N, C], device=dev) + 0.5
for name, fn in [('plain_bias_lrelu', lambda: cg.conv3x3_fused(x, wp, C, bias=b, act=1, gain=1.41, clamp=256.0)),
                 ('dgrad_dot', lambda: cg.conv3x3_fused(x, wp, C, out_scale=s, dot_src=x))]:
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    e1.synchronize()
    print(f'   {name}: {e0.elapsed_time(e1) / 20:.4f} ms', flush=True)
