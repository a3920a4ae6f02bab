"""Training statistics: per-name moments [count, sum, sum of squares] accumulated on the device and
reduced across ranks on demand.

Public surface of SG3/torch_utils/training_stats.py (`init_multiprocessing` :34-51, `report` :55-99,
`report0` :103-109, `Collector` :113-230): the ADA heuristic (training_loop_mi_multimodal.py:373-376)
and the per-tick stats.jsonl (:461-469) read it.

Design (this build's own):
  * every statistic name owns one row of a per-device float64 table (`_Board`), rows in first-report
    order; `report` adds the value's three moments into that row in place: no host sync and, once the
    row exists, no allocation -- so reports inside a HIP-graph-captured phase replay correctly;
  * `Collector.update` drains ALL device tables in one pass into one `[rows, 3]` tensor, all-reduces it
    once across ranks, and folds it into a process-wide CPU cumulative table (numpy float64); each
    collector remembers the cumulative totals it saw last and exposes the difference.
As in the reference, every rank must report the same names in the same order (`report0` registers
the name on every rank).
"""
import re

import numpy as np
import torch

import dnnlib


class _Board:
    def __init__(self):
        self.rows = {}               # name -> row index
        self.tables = {}             # device -> float64 [capacity, 3]
        self.capacity = 256
        self.captured = False        # a HIP graph holds pointers into the tables: they may not be replaced
        self.total = np.zeros([0, 3], np.float64)   # cumulative moments after the last drain
        self.rank = 0
        self.sync_device = None
        self.synced = False

    def row(self, name):
        r = self.rows.get(name)
        if r is None:
            r = self.rows[name] = len(self.rows)
            if r >= self.capacity:           # grow every table (rows are registered by the eager warm-up step)
                if self.captured or (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
                    # captured graphs keep accumulating into the old tables: every later report (Loss/signs/real,
                    # which drives ADA's p, included) would be dropped silently
                    del self.rows[name]
                    raise RuntimeError(f'training_stats: statistic {name!r} is new after a HIP graph was captured '
                                       f'and the board is full ({self.capacity} rows); register it before capture')
                self.capacity *= 2
                for dev, t in self.tables.items():
                    g = torch.zeros([self.capacity, 3], dtype=torch.float64, device=dev)
                    g[:t.shape[0]].copy_(t)
                    self.tables[dev] = g
        return r

    def table(self, device):
        t = self.tables.get(device)
        if t is None:
            t = self.tables[device] = torch.zeros([self.capacity, 3], dtype=torch.float64, device=device)
        return t

    def drain(self):
        """Move every device's pending moments into the cumulative table (one all_reduce over ranks)."""
        n = len(self.rows)
        if n == 0:
            return self.total
        self.synced = True
        dev = self.sync_device if self.sync_device is not None else torch.device('cpu')
        acc = torch.zeros([n, 3], dtype=torch.float64, device=dev)
        for t in self.tables.values():
            acc.add_(t[:n].to(dev))
            t.zero_()
        if self.sync_device is not None:
            torch.distributed.all_reduce(acc)
        if self.total.shape[0] < n:
            self.total = np.concatenate([self.total, np.zeros([n - self.total.shape[0], 3])])
        self.total[:n] += acc.cpu().numpy()
        return self.total


_board = _Board()


def mark_captured():
    """A HIP graph that reports statistics has been captured: the device tables are fixed from now on."""
    _board.captured = True


def init_multiprocessing(rank, sync_device):
    """Call after init_process_group and before the first Collector.update (reference :34-51)."""
    assert not _board.synced, 'init_multiprocessing must precede the first Collector.update()'
    _board.rank = rank
    _board.sync_device = sync_device


def report(name, value):
    """Accumulate the moments of `value` (any scalar set) under `name`; returns `value` unchanged."""
    return _report(name, value, 0)


def report_sign(name, value):
    """report(name, value.sign()) -- on the device without materialising the sign.  When a caller has replaced
    `report` (tests that record the reported stream), the sign goes through the replacement."""
    if report is not _REPORT:
        report(name, torch.as_tensor(value).sign())
        return value
    return _report(name, value, 1)


def _report(name, value, mode):
    r = _board.row(name)
    v = torch.as_tensor(value)
    if v.numel() == 0:
        return value
    if v.is_cuda:     # one launch (sg2_moments) instead of flatten / square / sums / stack / cast / adds
        import sg2hip as _hip
        vf = v.detach().reshape(-1)
        if vf.dtype != torch.float32 or not vf.is_contiguous():
            vf = vf.float().contiguous()
        row = _board.table(v.device)[r]
        _hip.check(_hip.lib().sg2_moments(_hip.ptr(row), _hip.ptr(vf), vf.numel(), mode, _hip.stream_ptr(v.device)),
                   'sg2_moments')
        return value
    v = v.detach().flatten().float()
    if mode == 1:
        v = v.sign()
    moments = torch.stack([v.sum(), v.square().sum()]).double()
    row = _board.table(v.device)[r]
    row[1:].add_(moments)
    row[:1].add_(float(v.numel()))
    return value


_REPORT = report


def report0(name, value):
    """`report` on rank 0 only; the other ranks register the name with no scalars."""
    report(name, value if _board.rank == 0 else [])
    return value


class Collector:
    """Means / standard deviations of the reported scalars between the last two `update()` calls, for
    names matching `regex`.  With keep_previous, a name that received nothing keeps its last values."""

    def __init__(self, regex='.*', keep_previous=True):
        self._regex = re.compile(regex)
        self._keep_previous = keep_previous
        self._seen = {}      # name -> cumulative moments at the last update
        self._delta = {}     # name -> moments between the last two updates
        self.update()
        self._delta.clear()

    def names(self):
        return [n for n in _board.rows if self._regex.fullmatch(n)]

    def update(self):
        if not self._keep_previous:
            self._delta.clear()
        names = self.names()
        if not names:
            return
        total = _board.drain()
        for n in names:
            cur = total[_board.rows[n]].copy()
            d = cur - self._seen.get(n, 0.0)
            self._seen[n] = cur
            if d[0] != 0:
                self._delta[n] = d

    def _moments(self, name):
        assert self._regex.fullmatch(name)
        return self._delta.get(name, np.zeros(3))

    def num(self, name):
        return int(self._moments(name)[0])

    def mean(self, name):
        cnt, s, _ = self._moments(name)
        return float('nan') if int(cnt) == 0 else float(s / cnt)

    def std(self, name):
        cnt, s, sq = self._moments(name)
        if int(cnt) == 0 or not np.isfinite(s):
            return float('nan')
        if int(cnt) == 1:
            return 0.0
        m = s / cnt
        return float(np.sqrt(max(sq / cnt - m * m, 0.0)))

    def as_dict(self):
        return dnnlib.EasyDict({n: dnnlib.EasyDict(num=self.num(n), mean=self.mean(n), std=self.std(n))
                                for n in self.names()})

    def __getitem__(self, name):
        return self.mean(name)
