"""Loading network snapshots (drop-in for SG3/legacy.py:22-58 `load_network_pkl`).

A snapshot is the reference's `network-snapshot-<kimg>.pkl`: a pickle of dict(G, D, G_ema, augment_pipe,
training_set_kwargs) whose modules are persistent objects (torch_utils/persistence.py).  It is read with
`SnapshotUnpickler`, which admits only what such a file legitimately contains -- tensors and storages,
builtin containers, torch dtypes / devices, dnnlib.EasyDict, numpy arrays and the persistent-object
reconstructor -- and rebuilds every module from this build's classes (no embedded source is executed).
The reference's conversion of TensorFlow-era pickles (legacy.py:60-320) is out of scope: the Claro /
Pelvis runs write PyTorch pickles.
"""
import copy
import io
import pickle

import numpy as np
import torch

import dnnlib
from torch_utils import misc
from torch_utils import persistence


def _storage_from_bytes(b):
    # torch.storage._load_from_bytes without the unrestricted unpickler: the bytes are a torch.save of one
    # storage, which the weights-only loader reads
    return torch.load(io.BytesIO(b), weights_only=True)


class SnapshotUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ('collections', 'OrderedDict'), ('builtins', 'set'), ('builtins', 'frozenset'), ('builtins', 'slice'),
        ('builtins', 'range'), ('builtins', 'complex'),
        ('torch._utils', '_rebuild_tensor_v2'), ('torch._utils', '_rebuild_tensor'),
        ('torch._utils', '_rebuild_parameter'), ('torch._utils', '_rebuild_parameter_with_state'),
        ('torch', 'Size'), ('torch', 'device'), ('numpy', 'ndarray'), ('numpy', 'dtype'),
        ('numpy.core.multiarray', '_reconstruct'), ('numpy.core.multiarray', 'scalar'),
        ('numpy._core.multiarray', '_reconstruct'), ('numpy._core.multiarray', 'scalar'),
    }
    _TORCH_DTYPES = {'float16', 'float32', 'float64', 'bfloat16', 'int64', 'int32', 'uint8', 'bool'}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        if module == 'torch.storage' and name == '_load_from_bytes':
            return _storage_from_bytes
        if module == 'torch' and (name in self._TORCH_DTYPES or name.endswith('Storage')):
            return getattr(torch, name)
        if module == 'torch_utils.persistence' and name == '_reconstruct_persistent_obj':
            return persistence._reconstruct_persistent_obj
        if module == 'dnnlib.util' and name == 'EasyDict':
            return dnnlib.EasyDict
        if module == 'numpy' and name in ('float16', 'float32', 'float64', 'int64', 'int32', 'uint8', 'bool_'):
            return getattr(np, name)
        if module == 'dnnlib.tflib.network':
            raise pickle.UnpicklingError('TensorFlow-era network pickle: conversion is out of scope')
        raise pickle.UnpicklingError(f'snapshot refers to {module}.{name}: not part of a network snapshot; refused')


def load_network_pkl(f, force_fp16=False):
    """dict(G, D, G_ema, augment_pipe, training_set_kwargs) from an open snapshot file (reference :22-58)."""
    data = SnapshotUnpickler(f).load()
    if not isinstance(data, dict):
        raise pickle.UnpicklingError('not a network snapshot (expected a dict)')
    data.setdefault('training_set_kwargs', None)
    data.setdefault('augment_pipe', None)
    for key in ('G', 'D', 'G_ema'):
        assert isinstance(data[key], torch.nn.Module), key
    assert isinstance(data['training_set_kwargs'], (dict, type(None)))
    assert isinstance(data['augment_pipe'], (torch.nn.Module, type(None)))
    if force_fp16:
        for key in ('G', 'D', 'G_ema'):
            old = data[key]
            kwargs = copy.deepcopy(old.init_kwargs)
            fp16_kwargs = kwargs.get('synthesis_kwargs', kwargs)
            fp16_kwargs.num_fp16_res = 4
            fp16_kwargs.conv_clamp = 256
            if kwargs != old.init_kwargs:
                new = type(old)(**kwargs).eval().requires_grad_(False)
                misc.copy_params_and_buffers(old, new, require_all=True)
                data[key] = new
    return data


def save_network_pkl(path, G, D, G_ema, augment_pipe=None, training_set_kwargs=None, num_gpus=1):
    """network-snapshot pickle as the reference writes it (training_loop_mi_multimodal.py:420-434): CPU
    copies in eval mode, replicas checked for consistency and broadcast from rank 0 first."""
    data = dict(G=G, D=D, G_ema=G_ema, augment_pipe=augment_pipe,
                training_set_kwargs=dict(training_set_kwargs) if training_set_kwargs is not None else None)
    for key, value in list(data.items()):
        if isinstance(value, torch.nn.Module):
            value = copy.deepcopy(value).eval().requires_grad_(False)
            if num_gpus > 1:
                misc.check_ddp_consistency(value, ignore_regex=r'.*\.[^.]+_(avg|ema)')
                for t in misc.params_and_buffers(value):
                    torch.distributed.broadcast(t, src=0)
            data[key] = value.cpu()
    if path is not None:
        with open(path, 'wb') as f:
            pickle.dump(data, f)
    return data
