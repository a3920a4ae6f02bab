import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'gan-track_amd')
for p in (ROOT, PKG, os.path.join(ROOT, 'tests', 'golden')):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs on the GPU box)')
    config.addinivalue_line('markers', 'slow: long-running')


# Unit-level files first, whole-iteration files last: a failure under -x then stops the run after the kernel
# tests have reported, not before them.
_ORDER = ['test_capi', 'test_oracle_golden', 'test_loss_host', 'test_trainer_shell', 'test_dist_gloo', 'test_ops_gpu',
          'test_deterministic_gpu', 'test_train_gpu', 'test_trainer_gpu', 'test_training_loop_gpu', 'test_bench_gpu', 'test_config_gpu']


def _rank(item):
    mod = os.path.splitext(os.path.basename(str(item.fspath)))[0]
    return _ORDER.index(mod) if mod in _ORDER else len(_ORDER)


def pytest_collection_modifyitems(config, items):
    items.sort(key=_rank)     # stable: the order inside a file is kept
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason='no GPU in this container')
    for item in items:
        if 'gpu' in item.keywords:
            item.add_marker(skip)
