"""Optimiser step and G_ema update of the training iteration as multi-tensor HIP launches.

Reference: SG3/training/training_loop_mi_multimodal.py:341-351 (flat gradient, all_reduce, /N, nan_to_num,
torch.optim.Adam(betas=(0, 0.99), eps=1e-8) step) and :358-366 (G_ema = G.lerp(G_ema, beta)).

`FlatAdam` keeps torch.optim.Adam's arithmetic and its per-parameter state semantics (a parameter
without a gradient in a phase is skipped and its step count does not advance -- Gmain and Greg share one
optimiser, so their counts differ), but steps a whole module in ONE launch of sg2_adam_multi, reading the
exchanged flat gradient directly: the reference's cat / divide / nan_to_num / split passes and torch's
foreach Adam kernels are a single HBM pass.  `ema_lerp` updates every G_ema tensor in one sg2_lerp_multi.
"""
import math

import torch

import sg2hip

CHUNK = 4096      # elements per work item (csrc/misc.hip SEG_CHUNK)


def _block_table(sizes, device):
    """(segment << 40) | start for every 4096-element chunk of every segment."""
    entries = [(s << 40) | start for s, n in enumerate(sizes) for start in range(0, n, CHUNK)]
    assert len(sizes) < (1 << 23) and max(sizes, default=0) < (1 << 40)
    return torch.tensor(entries, dtype=torch.int64).to(device), len(entries)


class FlatAdam:
    """torch.optim.Adam (no weight decay, amsgrad off) for the parameters of one module, stepped from a
    flat gradient whose layout the trainer's GradExchange defines."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False):
        if weight_decay != 0 or amsgrad:
            raise ValueError('FlatAdam implements Adam without weight decay / amsgrad (the reference\'s setting)')
        self.params = list(params)
        self.param_groups = [dict(params=self.params, lr=float(lr), betas=tuple(float(b) for b in betas),
                                  eps=float(eps))]
        self.steps = [0] * len(self.params)
        self.exp_avg = self.exp_avg_sq = None
        self._tables = {}

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    def step_flat(self, flat, offsets, part, grad_scale=1.0, write_grad=True, tag=None):
        """One Adam step of the parameters `part` (indices into self.params, those with a gradient this
        phase) from `flat`, where parameter i's gradient is flat[offsets[i] : offsets[i] + numel]."""
        if not part:
            return
        self.prepare(flat, offsets, part, tag)
        self.launch(flat, part, grad_scale, write_grad, tag)

    def _table(self, flat, offsets, part, tag=None):
        """Per (phase tag, participation set): segment table, chunk table and the device buffer of the step
        scalars.  Keyed by the phase as well: two phases sharing this optimiser (Gmain / Greg) may one day have
        the same participation set, and a step replays both phase graphs after staging both phases' scalars --
        one shared buffer would hand the first replay the second phase's bias corrections."""
        key = (tag, tuple(part))
        tab = self._tables.get(key)
        if tab is None:
            dev = flat.device
            seg = torch.tensor([[self.params[i].data_ptr(), offsets[i], self.params[i].numel()] for i in part],
                               dtype=torch.int64).to(dev)
            blocks, nb = _block_table([self.params[i].numel() for i in part], dev)
            coef = torch.zeros([2 * len(part)], dtype=torch.float32, device=dev)
            tab = self._tables[key] = (seg, blocks, nb, coef)
        return tab

    def prepare(self, flat, offsets, part, tag=None):
        """Advance the step counts of `part` and write torch.optim.Adam's step scalars into the set's device
        buffer (an asynchronous copy on the current stream, ordered before the launch that reads it -- which
        may be a replayed HIP graph)."""
        g = self.param_groups[0]
        lr, (b1, b2) = g['lr'], g['betas']
        if self.exp_avg is None:
            self.exp_avg = torch.zeros_like(flat)
            self.exp_avg_sq = torch.zeros_like(flat)
        coef_dev = self._table(flat, offsets, part, tag)[3]
        coef = []
        for i in part:           # torch.optim.Adam's scalars, computed in double as torch does
            self.steps[i] += 1
            s = self.steps[i]
            coef += [lr / (1 - b1 ** s), math.sqrt(1 - b2 ** s)]
        coef_dev.copy_(torch.tensor(coef, dtype=torch.float32).pin_memory(), non_blocking=True)

    def launch(self, flat, part, grad_scale=1.0, write_grad=True, tag=None):
        """The sg2_adam_multi launch of a prepared set (capturable: every operand is a persistent buffer)."""
        g = self.param_groups[0]
        (b1, b2), eps = g['betas'], g['eps']
        seg, blocks, nb, coef = self._tables[(tag, tuple(part))]
        L = sg2hip.lib()
        sg2hip.check(L.sg2_adam_multi(sg2hip.ptr(seg), sg2hip.ptr(coef), sg2hip.ptr(blocks), nb, sg2hip.ptr(flat),
                                      sg2hip.ptr(self.exp_avg), sg2hip.ptr(self.exp_avg_sq), b1, b2, eps,
                                      float(grad_scale), int(write_grad), sg2hip.stream_ptr(flat.device)),
                     'sg2_adam_multi')


class EmaLerp:
    """G_ema parameters <- G.lerp(G_ema, beta) in one sg2_lerp_multi launch; G_ema buffers <- G buffers."""

    def __init__(self, G_ema, G):
        self.dst = [p for p in G_ema.parameters()]
        self.src = [p for p in G.parameters()]
        self.bdst = [b for b in G_ema.buffers()]
        self.bsrc = [b for b in G.buffers()]
        assert [p.shape for p in self.dst] == [p.shape for p in self.src]
        assert all(p.dtype == torch.float32 and p.is_contiguous() for p in self.dst + self.src)
        dev = self.dst[0].device
        self.seg = torch.tensor([[d.data_ptr(), s.data_ptr(), d.numel()] for d, s in zip(self.dst, self.src)],
                                dtype=torch.int64).to(dev)
        self.blocks, self.nb = _block_table([d.numel() for d in self.dst], dev)

    def __call__(self, beta):
        dev = self.dst[0].device
        sg2hip.check(sg2hip.lib().sg2_lerp_multi(sg2hip.ptr(self.seg), sg2hip.ptr(self.blocks), self.nb,
                                                 float(beta), sg2hip.stream_ptr(dev)), 'sg2_lerp_multi')
        if self.bdst:
            torch._foreach_copy_(self.bdst, self.bsrc)


def fused_adam_ok(opt_kwargs, device):
    """The HIP optimiser serves the reference's optimiser class (torch.optim.Adam) on a ROCm device; any
    other class (or CPU host logic in the gloo tests) is constructed by name as the reference does."""
    return device is not None and torch.device(device).type == 'cuda' and \
        opt_kwargs.get('class_name') == 'torch.optim.Adam'

