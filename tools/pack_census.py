"""Which weight packs the training step still makes one launch each (GPU, eager): wraps
torch_utils/ops/conv2d_gradfix._pack_raw (the per-call sg2_pack_weight path, taken when a pack misses the phase's
pre-packed plan) and records per call site (the first networks/loss frames of the stack) the weight's shape,
dtype, pack form and whether it is a parameter (view).  Prints the counts per step over one 16-step cycle.
Usage: python tools/pack_census.py [bench args]"""
import os
import sys
import traceback
from collections import Counter

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402
from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

calls = Counter()
active = [False]
orig = cg._pack_raw


def site():
    fr = [f for f in traceback.extract_stack()[:-2] if 'gan-track_amd' in f.filename and 'conv2d_gradfix' not in f.filename]
    return ' < '.join(f'{os.path.basename(f.filename)}:{f.lineno}({f.name})' for f in fr[-3:][::-1])


def wrapped(w, a_dim, dtype, flip, scale):
    if active[0]:
        par = isinstance(w, torch.nn.Parameter) or isinstance(getattr(w, '_base', None), torch.nn.Parameter)
        calls[(site(), tuple(w.shape), str(dtype or w.dtype).replace('torch.', ''), a_dim, bool(flip),
               'param' if par else 'tensor', cg._pack_cache is not None)] += 1
    return orig(w, a_dim, dtype, flip, scale)


cg._pack_raw = wrapped
sys.argv = [sys.argv[0], '--graphs', 'off', '--no-cpu-baseline'] + sys.argv[1:]
args = bench.parse()
dev = torch.device('cuda', 0)
tr = bench.build(args, dev, 0, 1)
real, real_c = bench.make_inputs(args, dev, 0)
for _ in range(17):
    bench.one_step(tr, args, dev, real, real_c)
torch.cuda.synchronize()
active[0] = True
for _ in range(16):
    bench.one_step(tr, args, dev, real, real_c)
torch.cuda.synchronize()
print(f'single packs: {sum(calls.values()) / 16:.2f} per step')
for k, v in calls.most_common(60):
    print(f'{v / 16:6.2f}/step  {k}')
