"""Where the step's torch (non-HIP-kernel) launches come from (GPU, eager): records every aten op that one
16-iteration cycle dispatches, keyed by the op and its origin -- the autograd node running it (backward)
or the innermost frames of this repo's code (forward) -- and prints the most frequent per step.
Usage: python tools/glue_census.py [phase]   (phase: count only that loss phase, e.g. Greg)"""
import os
import sys
import traceback
from collections import Counter

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402

VIEWS = {'view', 'as_strided', 'reshape', 't', 'transpose', 'permute', 'expand', 'slice', 'select', 'detach',
         'alias', 'unsqueeze', 'squeeze', '_reshape_alias', 'empty', 'empty_strided', 'empty_like', 'unbind',
         'split', 'split_with_sizes', 'narrow', 'unfold', 'lift_fresh', 'resolve_conj', 'resolve_neg', 'new_empty',
         'new_empty_strided', '_unsafe_view', 'numpy_T', 'mT', 'expand_as', 'view_as', 'set_', 'clone', 'is_nonzero',
         'item', '_local_scalar_dense', 'resize_', 'contiguous'}
counts = Counter()
big = Counter()      # ops over >= 1M-element tensors: (op, origin, shape, dtype) -> count


CUR = {'phase': None}


class Census(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        if name not in VIEWS and (ONLY is None or CUR['phase'] == ONLY):
            node = torch._C._current_autograd_node()
            if node is not None:
                origin = 'bwd ' + node.name()
            else:
                fr = [f for f in traceback.extract_stack() if 'gan-track_amd' in f.filename]
                origin = ' <- '.join(f'{f.filename.split("gan-track_amd/")[-1]}:{f.lineno}' for f in fr[-2:][::-1])
            counts[(name, origin)] += 1
            t = next((a for a in args if isinstance(a, torch.Tensor)), None)
            if t is not None and t.numel() >= (1 << 20):
                big[(name, origin, tuple(t.shape), str(t.dtype).split('.')[-1])] += 1
        return func(*args, **(kwargs or {}))


ONLY = sys.argv[1] if len(sys.argv) > 1 else None
sys.argv = [sys.argv[0], '--graphs', 'off', '--no-cpu-baseline']
args = bench.parse()
dev = torch.device('cuda', 0)
tr = bench.build(args, dev, 0, 1)
_orig_acc = type(tr.loss).accumulate_gradients


def _acc(self, *a, **k):
    CUR['phase'] = k.get('phase', a[0] if a else None)
    try:
        return _orig_acc(self, *a, **k)
    finally:
        CUR['phase'] = None


type(tr.loss).accumulate_gradients = _acc
real, real_c = bench.make_inputs(args, dev, 0)
for _ in range(2):
    bench.one_step(tr, args, dev, real, real_c)
torch.cuda.synchronize()
with Census():
    for _ in range(16):
        bench.one_step(tr, args, dev, real, real_c)
torch.cuda.synchronize()
print(f'{sum(counts.values()) / 16:.0f} non-view aten ops per step')
for (op, origin), n in counts.most_common(70):
    print(f'{n / 16:7.1f}/step {op:18s} {origin[:160]}')
print('\nops on >= 1M-element tensors (bytes moved dominate the glue time):')
for (op, origin, shp, dt), n in big.most_common(40):
    print(f'{n / 16:7.1f}/step {op:14s} {dt:8s} {str(shp):24s} {origin[:120]}')
