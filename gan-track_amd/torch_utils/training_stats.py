"""Cross-rank scalar statistics (the ADA heuristic reads 'Loss/signs/real' through it).

Same API and semantics as SG3/torch_utils/training_stats.py: `report`/`report0` accumulate
[count, sum, sum of squares] per name per device without host syncs (:55-99); `Collector.update`
sums the deltas of all names in ONE all_reduce of a [num_names, 3] float64 tensor (:234-266)."""
import re

import numpy as np
import torch

import dnnlib

_num_moments = 3
_reduce_dtype = torch.float32
_counter_dtype = torch.float64
_rank = 0
_sync_device = None
_sync_called = False
_counters = {}     # name -> device -> tensor[3]
_cumulative = {}   # name -> cpu tensor[3]


def init_multiprocessing(rank, sync_device):
    global _rank, _sync_device
    assert not _sync_called
    _rank = rank
    _sync_device = sync_device


def report(name, value):
    if name not in _counters:
        _counters[name] = {}
    elems = torch.as_tensor(value)
    if elems.numel() == 0:
        return value
    elems = elems.detach().flatten().to(_reduce_dtype)
    moments = torch.stack([torch.ones_like(elems).sum(), elems.sum(), elems.square().sum()])
    assert moments.ndim == 1 and moments.shape[0] == _num_moments
    moments = moments.to(_counter_dtype)
    dev = moments.device
    if dev not in _counters[name]:
        _counters[name][dev] = torch.zeros_like(moments)
    _counters[name][dev].add_(moments)
    return value


def report0(name, value):
    report(name, value if _rank == 0 else [])
    return value


class Collector:
    def __init__(self, regex='.*', keep_previous=True):
        self._regex = re.compile(regex)
        self._keep_previous = keep_previous
        self._cumulative = {}
        self._moments = {}
        self.update()
        self._moments.clear()

    def names(self):
        return [n for n in _counters if self._regex.fullmatch(n)]

    def update(self):
        if not self._keep_previous:
            self._moments.clear()
        for name, cum in _sync(self.names()):
            if name not in self._cumulative:
                self._cumulative[name] = torch.zeros([_num_moments], dtype=_counter_dtype)
            delta = cum - self._cumulative[name]
            self._cumulative[name].copy_(cum)
            if float(delta[0]) != 0:
                self._moments[name] = delta

    def _get_delta(self, name):
        assert self._regex.fullmatch(name)
        if name not in self._moments:
            self._moments[name] = torch.zeros([_num_moments], dtype=_counter_dtype)
        return self._moments[name]

    def num(self, name):
        return int(self._get_delta(name)[0])

    def mean(self, name):
        d = self._get_delta(name)
        return float('nan') if int(d[0]) == 0 else float(d[1] / d[0])

    def std(self, name):
        d = self._get_delta(name)
        if int(d[0]) == 0 or not np.isfinite(float(d[1])):
            return float('nan')
        if int(d[0]) == 1:
            return 0.0
        m = float(d[1] / d[0])
        return float(np.sqrt(max(float(d[2] / d[0]) - m * m, 0)))

    def as_dict(self):
        out = dnnlib.EasyDict()
        for n in self.names():
            out[n] = dnnlib.EasyDict(num=self.num(n), mean=self.mean(n), std=self.std(n))
        return out

    def __getitem__(self, name):
        return self.mean(name)


def _sync(names):
    if len(names) == 0:
        return []
    global _sync_called
    _sync_called = True
    device = _sync_device if _sync_device is not None else torch.device('cpu')
    deltas = []
    for name in names:
        d = torch.zeros([_num_moments], dtype=_counter_dtype, device=device)
        for c in _counters[name].values():
            d.add_(c.to(device))
            c.zero_()
        deltas.append(d)
    deltas = torch.stack(deltas)
    if _sync_device is not None:
        torch.distributed.all_reduce(deltas)
    deltas = deltas.cpu()
    for i, name in enumerate(names):
        if name not in _cumulative:
            _cumulative[name] = torch.zeros([_num_moments], dtype=_counter_dtype)
        _cumulative[name].add_(deltas[i])
    return [(n, _cumulative[n]) for n in names]
