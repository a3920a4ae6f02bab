"""Metric registry of the training loop (SG3/metrics/metric_main_mi_multimodal.py:27-95): calc_metric,
report_metric (metric-<modality>-<metric>.jsonl), and the FID metrics the Claro / Pelvis runs use."""
import json
import os
import time

import torch

import dnnlib
from . import metric_utils
from . import frechet_inception_distance

_metric_dict = {}


def register_metric(fn):
    assert callable(fn)
    _metric_dict[fn.__name__] = fn
    return fn


def is_valid_metric(metric):
    return metric in _metric_dict


def list_valid_metrics():
    return list(_metric_dict.keys())


def calc_metric(metric, **kwargs):
    assert is_valid_metric(metric)
    opts = metric_utils.MetricOptions(**kwargs)
    t0 = time.time()
    results = _metric_dict[metric](opts)
    total = time.time() - t0
    for key, value in list(results.items()):
        if opts.num_gpus > 1:
            v = torch.as_tensor(value, dtype=torch.float64, device=opts.device)
            torch.distributed.broadcast(v, src=0)
            value = float(v.cpu())
        results[key] = value
    return dnnlib.EasyDict(results=dnnlib.EasyDict(results), metric=metric, total_time=total,
                           total_time_str=dnnlib.util.format_time(total), num_gpus=opts.num_gpus)


def report_metric(result_dict, mode, run_dir=None, snapshot_pkl=None):
    metric = result_dict['metric']
    result_dict['mode'] = mode
    assert is_valid_metric(metric)
    if run_dir is not None and snapshot_pkl is not None:
        snapshot_pkl = os.path.relpath(snapshot_pkl, run_dir)
    line = json.dumps(dict(result_dict, snapshot_pkl=snapshot_pkl, timestamp=time.time()))
    print(line)
    if run_dir is not None and os.path.isdir(run_dir):
        with open(os.path.join(run_dir, f'metric-{mode}-{metric}.jsonl'), 'at') as f:
            f.write(line + '\n')


@register_metric
def fid50k_full(opts):
    opts.dataset_kwargs.update(max_size=None, xflip=False)
    return dict(fid50k_full=frechet_inception_distance.compute_fid(opts, max_real=None, num_gen=50000))


@register_metric
def fid50k(opts):
    opts.dataset_kwargs.update(max_size=None)
    return dict(fid50k=frechet_inception_distance.compute_fid(opts, max_real=50000, num_gen=50000))
