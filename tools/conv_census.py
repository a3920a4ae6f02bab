"""Which conv launches the training step spends its conv time on (GPU, eager): wraps the conv entry
points of torch_utils/ops/conv2d_gradfix.py, times every call with HIP events (synchronising -- the
times are per-call kernel times, not the overlapped step), and prints the total per (entry, shape) over
16 iterations (one full Greg/Dreg cycle) divided by 16.  Usage: python tools/conv_census.py [bench args]"""
import os
import sys
from collections import defaultdict

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

stats = defaultdict(lambda: [0, 0.0])
active = [False]


def wrap(name, fn, key):
    def w(*a, **k):
        if not active[0]:
            return fn(*a, **k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn(*a, **k)
        e1.record()
        e1.synchronize()
        s = stats[(name,) + key(*a, **k)]
        s[0] += 1
        s[1] += e0.elapsed_time(e1)
        return out
    return w


def shp(t):
    return tuple(t.shape) + (str(t.dtype).replace('torch.', ''),)


cg._conv_raw = wrap('conv', cg._conv_raw, lambda x, wp, cout, oh, ow, kh, kw, s, p, tr: shp(x) + (cout, oh, ow, kh, s, 'T' if tr else ''))
def _fused_key(x, wp, cout, oh, ow, kh, kw, s, p, transpose=False, **k):
    plain = all(k.get(n) is None for n in ('out_scale', 'noise', 'bias', 'residual', 'dot_src')) and \
        k.get('act', 0) == 0 and k.get('gain', 1.0) == 1.0 and k.get('clamp', -1.0) < 0 and not k.get('aux_mode', 0)
    be = 'up2' if plain and cg._up2_ok(x, cout, oh, ow, kh, kw, s, p, transpose) else \
        ('generic16' if x.dtype != torch.float32 else 'generic32')
    epi = '+'.join(n for n in ('in_scale', 'out_scale', 'bias', 'residual', 'dot_src') if k.get(n) is not None)
    return shp(x) + (cout, oh, ow, kh, s, 'T' if transpose else '', be, epi)


cg.conv_fused = wrap('conv_fused', cg.conv_fused, _fused_key)
cg._wgrad_raw = wrap('wgrad', cg._wgrad_raw, lambda g, x, kh, kw, s, p, **k: shp(g) + tuple(x.shape[1:]) + (kh, s))
cg.conv3x3_fused = wrap('conv3x3', cg.conv3x3_fused, lambda x, wp, cout, **k: shp(x) + (cout,))

sys.argv = [sys.argv[0], '--graphs', 'off', '--no-cpu-baseline'] + sys.argv[1:]
args = bench.parse()
dev = torch.device('cuda', 0)
tr = bench.build(args, dev, 0, 1)
real, real_c = bench.make_inputs(args, dev, 0)
for _ in range(2):
    bench.one_step(tr, args, dev, real, real_c)
torch.cuda.synchronize()
active[0] = True
for _ in range(16):
    bench.one_step(tr, args, dev, real, real_c)
torch.cuda.synchronize()
tot = sum(v[1] for v in stats.values()) / 16
print(f'conv calls: {sum(v[0] for v in stats.values()) / 16:.1f} per step, {tot:.2f} ms per step (synchronous)')
fam = {}
for k, v in stats.items():
    b = k[-2] if k[0] == 'conv_fused' else k[0]
    fam[b] = fam.get(b, 0.0) + v[1] / 16
print('per backend (ms/step): ' + ', '.join(f'{b} {t:.2f}' for b, t in sorted(fam.items(), key=lambda kv: -kv[1])))
for k, v in sorted(stats.items(), key=lambda kv: -kv[1][1])[:80]:
    print(f'{v[1] / 16:7.3f} ms/step {v[0] / 16:5.2f}/step {v[1] / v[0] * 1e3:8.1f} us  {k}')
