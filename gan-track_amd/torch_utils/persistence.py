"""Snapshot persistence: the reference's pickle format, loaded without executing embedded code.

Format (SG3/torch_utils/persistence.py:35-130, version 6): an instance of a decorated class pickles as
`torch_utils.persistence._reconstruct_persistent_obj(meta)`, meta = {type: 'class', version: 6,
module_src: <source of the class's module>, class_name, state: <the instance __dict__, with the recorded
constructor arguments _init_args / _init_kwargs>}.  Snapshots written here have exactly that structure
(network-snapshot-*.pkl = pickle of dict(G, D, G_ema, augment_pipe, training_set_kwargs)).

Loading differs by design.  The reference exec()s `module_src` to rebuild the class.  Here
`_reconstruct_persistent_obj` resolves `class_name` to this build's decorated class of the same name,
constructs it from the recorded constructor arguments (the drop-in module API accepts the reference's),
and copies the pickled parameters and buffers in by name -- so the reference's snapshots and this
build's load alike, and nothing embedded in a pickle is executed.  Combined with legacy.SafeUnpickler
(which admits only tensors, containers and these reconstructors) a snapshot cannot run code.
The classes served are the StyleGAN2 networks and the ADA pipe; a StyleGAN3 pickle is refused.
"""
import copy
import inspect
import sys

import torch

import dnnlib

_version = 6
_decorators = set()
_registry = {}          # class name -> decorated class
_module_src = {}        # module -> source text


def persistent_class(orig_class):
    """Class decorator: records constructor arguments and pickles in the reference's persistent format."""
    assert isinstance(orig_class, type)
    if is_persistent(orig_class):
        return orig_class
    module = sys.modules[orig_class.__module__]

    class Decorator(orig_class):
        _orig_module = module
        _orig_class_name = orig_class.__name__

        def __init__(self, *args, **kwargs):
            super().__init__(*args, **kwargs)
            self._init_args = copy.deepcopy(args)
            self._init_kwargs = copy.deepcopy(kwargs)

        @property
        def init_args(self):
            return copy.deepcopy(self._init_args)

        @property
        def init_kwargs(self):
            return dnnlib.EasyDict(copy.deepcopy(self._init_kwargs))

        def __deepcopy__(self, memo):
            # a plain member-wise copy (devices kept); only pickling goes through the persistent format
            obj = type(self).__new__(type(self))
            memo[id(self)] = obj
            for k, v in self.__dict__.items():
                obj.__dict__[k] = copy.deepcopy(v, memo)
            return obj

        def __reduce__(self):
            fields = list(super().__reduce__())
            fields += [None] * max(3 - len(fields), 0)
            if fields[0] is not _reconstruct_persistent_obj:
                meta = dict(type='class', version=_version, module_src=_source_of(self._orig_module),
                            class_name=self._orig_class_name, state=fields[2])
                fields = [_reconstruct_persistent_obj, (meta,), None] + fields[3:]
            return tuple(fields)

    Decorator.__name__ = orig_class.__name__
    Decorator.__qualname__ = orig_class.__qualname__
    _decorators.add(Decorator)
    _registry.setdefault(orig_class.__name__, Decorator)
    return Decorator


def is_persistent(obj):
    try:
        if obj in _decorators:
            return True
    except TypeError:
        pass
    return type(obj) in _decorators


def _source_of(module):
    src = _module_src.get(module)
    if src is None:
        src = _module_src[module] = inspect.getsource(module)
    return src


def _resolve(class_name, module_src):
    if 'class SynthesisInput' in (module_src or '') or 'filtered_lrelu' in (module_src or ''):
        raise pickle_error(f'{class_name}: a StyleGAN3 network (networks_stylegan3) -- out of scope, only the '
                           'StyleGAN2 configuration is served')
    cls = _registry.get(class_name)
    if cls is None:
        _import_network_modules()
        cls = _registry.get(class_name)
    if cls is None:
        raise pickle_error(f'no class {class_name!r} in this build')
    return cls


def _import_network_modules():
    import training.networks_stylegan2  # noqa: F401  (registers the decorated classes)
    import training.augment_mi  # noqa: F401


def pickle_error(msg):
    import pickle
    return pickle.UnpicklingError(msg)


def _tensors_of(state, prefix=''):
    """name -> tensor for the parameters / buffers held (recursively) by a pickled module state."""
    out = {}
    for kind in ('_parameters', '_buffers'):
        for n, t in (state.get(kind) or {}).items():
            if t is not None:
                out[prefix + n] = t
    for n, m in (state.get('_modules') or {}).items():
        if isinstance(m, torch.nn.Module):
            for k, t in list(m.named_parameters()) + list(m.named_buffers()):
                out[f'{prefix}{n}.{k}'] = t
    return out


def _reconstruct_persistent_obj(meta):
    """Unpickling hook (same name and signature as the reference's): build this build's class from the
    recorded constructor arguments, then load the pickled tensors by name."""
    meta = dnnlib.EasyDict(meta)
    if meta.get('type') != 'class' or meta.get('version') != _version:
        raise pickle_error(f'unsupported persistent object (type {meta.get("type")}, version {meta.get("version")})')
    state = dict(meta.state or {})
    cls = _resolve(meta.class_name, meta.get('module_src'))
    args, kwargs = state.get('_init_args', ()), dict(state.get('_init_kwargs', {}))
    obj = cls(*args, **kwargs)
    want = dict(list(obj.named_parameters()) + list(obj.named_buffers()))
    have = _tensors_of(state)
    with torch.no_grad():
        for name, t in have.items():
            if name not in want:
                continue
            dst = want[name]
            if tuple(dst.shape) != tuple(t.shape):
                raise pickle_error(f'{meta.class_name}.{name}: shape {tuple(t.shape)} vs {tuple(dst.shape)}')
            dst.copy_(t.detach().to(dst.dtype))
    missing = [n for n in want if n not in have]
    if missing and any(not n.endswith(('resample_filter', 'Hz_geom', 'Hz_fbank')) for n in missing):
        raise pickle_error(f'{meta.class_name}: snapshot lacks {missing[:4]}')
    obj.train(bool(state.get('training', True)))
    return obj
