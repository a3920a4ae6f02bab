"""Metric registry of the training loop.  Drop-in for SG3/metrics/metric_main_mi_multimodal.py:27-95: the module
keeps the reference's entry points (register_metric, is_valid_metric, list_valid_metrics, calc_metric,
report_metric) and its output contract (one JSON line per evaluation appended to
<run_dir>/metric-<modality>-<metric>.jsonl); the FID metrics are the two the Claro / Pelvis runs name."""
import json
import os
import time

import torch

import dnnlib
from . import metric_utils
from . import frechet_inception_distance


class _Registry:
    """Metric name -> function(opts) -> {result name: float}; insertion-ordered."""

    def __init__(self):
        self.fns = {}

    def add(self, fn):
        if not callable(fn):
            raise AssertionError(f'metric {fn!r} is not callable')
        self.fns[fn.__name__] = fn
        return fn

    def check(self, name):
        if name not in self.fns:
            raise AssertionError(f'unknown metric {name!r}; valid: {sorted(self.fns)}')
        return self.fns[name]


_REGISTRY = _Registry()
register_metric = _REGISTRY.add


def is_valid_metric(metric):
    return metric in _REGISTRY.fns


def list_valid_metrics():
    return list(_REGISTRY.fns)


def _rank0_value(value, opts):
    """Every rank reports rank 0's number (the detector statistics are only complete there)."""
    if opts.num_gpus <= 1:
        return value
    t = torch.tensor(float(value), dtype=torch.float64, device=opts.device)
    torch.distributed.broadcast(t, src=0)
    return float(t.item())


def calc_metric(metric, **kwargs):
    """Evaluate one registered metric; returns {results, metric, total_time, total_time_str, num_gpus}."""
    fn = _REGISTRY.check(metric)
    opts = metric_utils.MetricOptions(**kwargs)
    start = time.time()
    raw = fn(opts)
    elapsed = time.time() - start
    results = dnnlib.EasyDict({name: _rank0_value(v, opts) for name, v in raw.items()})
    return dnnlib.EasyDict(results=results, metric=metric, total_time=elapsed,
                           total_time_str=dnnlib.util.format_time(elapsed), num_gpus=opts.num_gpus)


def report_metric(result_dict, mode, run_dir=None, snapshot_pkl=None):
    """Print the evaluation as one JSON line and append it to the run's per-modality metric log."""
    _REGISTRY.check(result_dict['metric'])
    result_dict['mode'] = mode
    rel = os.path.relpath(snapshot_pkl, run_dir) if (run_dir is not None and snapshot_pkl is not None) else snapshot_pkl
    record = dict(result_dict)
    record.update(snapshot_pkl=rel, timestamp=time.time())
    text = json.dumps(record)
    print(text)
    if run_dir is None or not os.path.isdir(run_dir):
        return
    path = os.path.join(run_dir, 'metric-%s-%s.jsonl' % (mode, result_dict['metric']))
    with open(path, 'at') as log:
        log.write(text + '\n')


def _fid(opts, name, max_real, xflip):
    """FID against all (max_real None) or 50k real images, 50k generated."""
    opts.dataset_kwargs.update(max_size=None)
    if xflip is not None:
        opts.dataset_kwargs.update(xflip=xflip)
    return {name: frechet_inception_distance.compute_fid(opts, max_real=max_real, num_gen=50000)}


@register_metric
def fid50k_full(opts):
    return _fid(opts, 'fid50k_full', None, False)


@register_metric
def fid50k(opts):
    return _fid(opts, 'fid50k', 50000, None)
