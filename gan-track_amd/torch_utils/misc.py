"""Utilities of the training path, mirroring SG3/torch_utils/misc.py (constant cache :20-40,
nan_to_num :45, assert_shape :82-95, profiled_function :100-105, InfiniteSampler :111-142,
parameter helpers :147-162, check_ddp_consistency :180-191, print_module_summary :196-266)."""
import contextlib
import re
import warnings

import numpy as np
import torch

import dnnlib

_constant_cache = {}


def constant(value, shape=None, dtype=None, device=None, memory_format=None):
    value = np.asarray(value)
    shape = tuple(shape) if shape is not None else None
    dtype = dtype if dtype is not None else torch.get_default_dtype()
    device = device if device is not None else torch.device('cpu')
    memory_format = memory_format if memory_format is not None else torch.contiguous_format
    key = (value.shape, value.dtype, value.tobytes(), shape, dtype, device, memory_format)
    t = _constant_cache.get(key)
    if t is None:
        t = torch.as_tensor(value.copy(), dtype=dtype, device=device)
        if shape is not None:
            t, _ = torch.broadcast_tensors(t, torch.empty(shape))
        t = t.contiguous(memory_format=memory_format)
        _constant_cache[key] = t
    return t


nan_to_num = torch.nan_to_num
symbolic_assert = torch._assert


@contextlib.contextmanager
def suppress_tracer_warnings():
    flt = ('ignore', None, torch.jit.TracerWarning, None, 0)
    warnings.filters.insert(0, flt)
    yield
    warnings.filters.remove(flt)


def assert_shape(tensor, ref_shape):
    if tensor.ndim != len(ref_shape):
        raise AssertionError(f'Wrong number of dimensions: got {tensor.ndim}, expected {len(ref_shape)}')
    for idx, (size, ref) in enumerate(zip(tensor.shape, ref_shape)):
        if ref is not None and int(size) != int(ref):
            raise AssertionError(f'Wrong size for dimension {idx}: got {size}, expected {ref}')


def profiled_function(fn):
    def wrapper(*args, **kwargs):
        with torch.autograd.profiler.record_function(fn.__name__):
            return fn(*args, **kwargs)
    wrapper.__name__ = fn.__name__
    return wrapper


class InfiniteSampler(torch.utils.data.Sampler):
    """Endless shuffled index stream; rank r yields every num_replicas-th index starting at r.
    Window shuffle as in the reference (misc.py:111-142) so the sample order matches it."""

    def __init__(self, dataset, rank=0, num_replicas=1, shuffle=True, seed=0, window_size=0.5):
        assert len(dataset) > 0 and num_replicas > 0 and 0 <= rank < num_replicas and 0 <= window_size <= 1
        super().__init__()
        self.dataset, self.rank, self.num_replicas = dataset, rank, num_replicas
        self.shuffle, self.seed, self.window_size = shuffle, seed, window_size

    def __iter__(self):
        order = np.arange(len(self.dataset))
        rnd = None
        window = 0
        if self.shuffle:
            rnd = np.random.RandomState(self.seed)
            rnd.shuffle(order)
            window = int(np.rint(order.size * self.window_size))
        idx = 0
        while True:
            i = idx % order.size
            if idx % self.num_replicas == self.rank:
                yield order[i]
            if window >= 2:
                j = (i - rnd.randint(window)) % order.size
                order[i], order[j] = order[j], order[i]
            idx += 1


def params_and_buffers(module):
    return list(module.parameters()) + list(module.buffers())


def named_params_and_buffers(module):
    return list(module.named_parameters()) + list(module.named_buffers())


def copy_params_and_buffers(src_module, dst_module, require_all=False):
    src = dict(named_params_and_buffers(src_module))
    with torch.no_grad():
        for name, t in named_params_and_buffers(dst_module):
            assert (name in src) or (not require_all)
            if name in src:
                t.copy_(src[name].detach())


@contextlib.contextmanager
def ddp_sync(module, sync):
    if sync or not isinstance(module, torch.nn.parallel.DistributedDataParallel):
        yield
    else:
        with module.no_sync():
            yield


def check_ddp_consistency(module, ignore_regex=None):
    for name, t in named_params_and_buffers(module):
        full = type(module).__name__ + '.' + name
        if ignore_regex is not None and re.fullmatch(ignore_regex, full):
            continue
        t = t.detach()
        if t.is_floating_point():
            t = nan_to_num(t)
        other = t.clone()
        torch.distributed.broadcast(tensor=other, src=0)
        assert (t == other).all(), full


def print_module_summary(module, inputs, max_nesting=3, skip_redundant=True):
    entries = []
    depth = [0]

    def pre(_m, _i):
        depth[0] += 1

    def post(m, _i, out):
        depth[0] -= 1
        if depth[0] <= max_nesting:
            outs = list(out) if isinstance(out, (tuple, list)) else [out]
            entries.append(dnnlib.EasyDict(mod=m, outputs=[t for t in outs if isinstance(t, torch.Tensor)]))

    hooks = [m.register_forward_pre_hook(pre) for m in module.modules()]
    hooks += [m.register_forward_hook(post) for m in module.modules()]
    outputs = module(*inputs)
    for h in hooks:
        h.remove()
    seen = set()
    for e in entries:
        e.params = [t for t in e.mod.parameters() if id(t) not in seen]
        e.buffers = [t for t in e.mod.buffers() if id(t) not in seen]
        e.outs = [t for t in e.outputs if id(t) not in seen]
        seen |= {id(t) for t in e.params + e.buffers + e.outs}
    if skip_redundant:
        entries = [e for e in entries if e.params or e.buffers or e.outs]
    names = {m: n for n, m in module.named_modules()}
    rows = [[type(module).__name__, 'Parameters', 'Buffers', 'Output shape', 'Datatype'], ['---'] * 5]
    tp = tb = 0
    for e in entries:
        name = '<top-level>' if e.mod is module else names[e.mod]
        ps = sum(t.numel() for t in e.params)
        bs = sum(t.numel() for t in e.buffers)
        shapes = [str(list(t.shape)) for t in e.outputs] + ['-']
        dts = [str(t.dtype).split('.')[-1] for t in e.outputs] + ['-']
        rows.append([name + (':0' if len(e.outputs) >= 2 else ''), str(ps) if ps else '-', str(bs) if bs else '-',
                     shapes[0], dts[0]])
        for k in range(1, len(e.outputs)):
            rows.append([name + f':{k}', '-', '-', shapes[k], dts[k]])
        tp += ps
        tb += bs
    rows += [['---'] * 5, ['Total', str(tp), str(tb), '-', '-']]
    widths = [max(len(c) for c in col) for col in zip(*rows)]
    print()
    for r in rows:
        print('  '.join(c + ' ' * (w - len(c)) for c, w in zip(r, widths)))
    print()
    return outputs
