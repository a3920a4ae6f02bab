"""One StyleGAN2-ADA training iteration, data-parallel over ranks (one process per GPU).

This is the hot loop of SG3/training/training_loop_mi_multimodal.py:308-376, factored out so the
training loop, bench.py and the tests drive the same code:

    for phase in [Gmain, Greg(every 4), Dmain, Dreg(every 16)]:           (:326-336)
        zero_grad; module.requires_grad_(True); accumulate over batch_gpu chunks
        flat = cat(grads); all_reduce(flat, SUM); flat /= N; nan_to_num  (:341-350)
        Adam step                                                       (:351)
    G_ema = lerp(G, G_ema, beta)                                         (:358-366)
    every ada_interval: p += sign(E[sign(D(real))] - target) * B*I/(ada_kimg*1000)   (:373-376)

Data parallel on MI355X: the gradient exchange is RCCL (torch.distributed backend 'nccl') over
xGMI.  Gradients are exchanged in buckets of `bucket_mb` MiB; with `overlap=True` each bucket's
all_reduce is issued from a post-accumulate-grad hook during the LAST micro-batch's backward, so
the collectives run on RCCL's stream while the remaining backward kernels execute.  The reduction is
a SUM then /N, then nan_to_num(0, +-1e5) -- the reference's arithmetic, bucketed (fp32 summation
order differs only by rounding).
"""
import numpy as np
import torch

import dnnlib
from torch_utils import misc
from torch_utils import training_stats


class GradReducer:
    """Bucketed, optionally backward-overlapped, flat gradient all-reduce for one module."""

    def __init__(self, module, num_gpus, bucket_mb=32, overlap=True):
        self.params = [p for p in module.parameters()]
        self.num_gpus = num_gpus
        self.overlap = overlap and num_gpus > 1
        self.bucket_elems = max(1, int(bucket_mb * (1 << 20) // 4))
        self._hooks = []
        self._armed = False
        self._pending = []

    # Buckets follow reverse registration order (roughly the order backward produces gradients).
    def _buckets(self, params):
        buckets, cur, size = [], [], 0
        for p in reversed(params):
            cur.append(p)
            size += p.numel()
            if size >= self.bucket_elems:
                buckets.append(cur)
                cur, size = [], 0
        if cur:
            buckets.append(cur)
        return buckets

    def arm(self, expected=1):
        """Call before the last micro-batch: launch a bucket's all_reduce once every parameter in it
        has accumulated `expected` gradients (the number of backward passes of this micro-batch)."""
        if not self.overlap:
            return
        self._armed = True
        self._pending = []
        trainable = [p for p in self.params if p.requires_grad]
        self._bucket_of = {}
        self._ready = []
        self._bucket_list = self._buckets(trainable)
        for bi, b in enumerate(self._bucket_list):
            self._ready.append(0)
            for p in b:
                self._bucket_of[p] = bi
        self._launched = [False] * len(self._bucket_list)

        def hook(p):
            bi = self._bucket_of.get(p)
            if bi is None or p.grad is None:   # the hook also fires for structurally-zero (undefined) grads
                return
            self._ready[bi] += 1
            if self._ready[bi] == expected * len(self._bucket_list[bi]) and not self._launched[bi]:
                self._launch(bi)

        self._hooks = [p.register_post_accumulate_grad_hook(hook) for p in trainable]

    def _launch(self, bi):
        b = self._bucket_list[bi]
        flat = torch.cat([p.grad.flatten() for p in b])
        work = torch.distributed.all_reduce(flat, async_op=True)
        self._pending.append((b, flat, work))
        self._launched[bi] = True

    def finish(self):
        """Reduce whatever is not reduced yet, average, sanitise and write back into .grad."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        params = [p for p in self.params if p.grad is not None]
        if not params:
            return
        done = set()
        results = []
        for b, flat, work in self._pending:
            results.append((b, flat, work))
            done.update(id(p) for p in b)
        rest = [p for p in params if id(p) not in done]
        if rest:
            flat = torch.cat([p.grad.flatten() for p in rest])
            work = torch.distributed.all_reduce(flat, async_op=True) if self.num_gpus > 1 else None
            results.append((rest, flat, work))
        for b, flat, work in results:
            if work is not None:
                work.wait()
            if self.num_gpus > 1:
                flat /= self.num_gpus
            misc.nan_to_num(flat, nan=0, posinf=1e5, neginf=-1e5, out=flat)
            for p, g in zip(b, flat.split([p.numel() for p in b])):
                p.grad = g.reshape(p.shape)
        self._pending = []
        self._armed = False


class Trainer:
    def __init__(self, G, D, G_ema, loss, G_opt_kwargs, D_opt_kwargs, G_reg_interval=4, D_reg_interval=16,
                 batch_size=32, batch_gpu=32, num_gpus=1, rank=0, device=None, ema_kimg=10, ema_rampup=0.05,
                 augment_pipe=None, ada_target=None, ada_interval=4, ada_kimg=500, bucket_mb=32, overlap=True,
                 phase_timing=False, graphs=False):
        self.G, self.D, self.G_ema, self.loss = G, D, G_ema, loss
        self.batch_size, self.batch_gpu, self.num_gpus, self.rank = batch_size, batch_gpu, num_gpus, rank
        self.device = device
        self.ema_kimg, self.ema_rampup = ema_kimg, ema_rampup
        self.augment_pipe, self.ada_target = augment_pipe, ada_target
        self.ada_interval, self.ada_kimg = ada_interval, ada_kimg
        self.ada_stats = training_stats.Collector(regex='Loss/signs/real') \
            if (augment_pipe is not None and ada_target is not None) else None
        self.phases = []
        for name, module, opt_kwargs, reg_interval in [('G', G, G_opt_kwargs, G_reg_interval),
                                                       ('D', D, D_opt_kwargs, D_reg_interval)]:
            reducer = GradReducer(module, num_gpus, bucket_mb=bucket_mb, overlap=overlap)
            if reg_interval is None:
                opt = dnnlib.util.construct_class_by_name(params=module.parameters(), **opt_kwargs)
                self.phases.append(dnnlib.EasyDict(name=name + 'both', module=module, opt=opt, interval=1,
                                                   reducer=reducer))
            else:   # lazy regularisation (:248-255)
                ratio = reg_interval / (reg_interval + 1)
                kw = dnnlib.EasyDict(opt_kwargs)
                kw.lr = kw.lr * ratio
                kw.betas = [b ** ratio for b in kw.betas]
                opt = dnnlib.util.construct_class_by_name(module.parameters(), **kw)
                self.phases.append(dnnlib.EasyDict(name=name + 'main', module=module, opt=opt, interval=1,
                                                   reducer=reducer))
                self.phases.append(dnnlib.EasyDict(name=name + 'reg', module=module, opt=opt,
                                                   interval=reg_interval, reducer=reducer))
        for ph in self.phases:
            ph.start_event = ph.end_event = None
            if phase_timing and device is not None and device.type == 'cuda':
                ph.start_event = torch.cuda.Event(enable_timing=True)
                ph.end_event = torch.cuda.Event(enable_timing=True)
        self.cur_nimg = 0
        self.batch_idx = 0
        self.on_grads = None   # optional callback(phase_name, module) after the gradient exchange
        # HIP-graph mode: each phase's forward + backward (all micro-batches) is captured once and
        # replayed; the gradient exchange, the optimiser, EMA and ADA stay eager.  Capture the first
        # time a phase runs in graph mode -- run at least one eager step first so every lazily created
        # state (kernel attributes, statistics counters, cached constants) exists before capture.
        self.graphs = graphs
        self._graphs = {}

    def _accumulate(self, phase, phase_real_img, phase_real_c, phase_gen_z, phase_gen_c, arm):
        chunks = list(zip(phase_real_img, phase_real_c, phase_gen_z, phase_gen_c))
        for ci, (real_img, real_c, gen_z, gen_c) in enumerate(chunks):
            if arm and ci == len(chunks) - 1:
                phase.reducer.arm(expected=2 if phase.name in ('Dmain', 'Dboth') else 1)
            self.loss.accumulate_gradients(phase=phase.name, real_img=real_img, real_c=real_c, gen_z=gen_z,
                                           gen_c=gen_c, gain=phase.interval, cur_nimg=self.cur_nimg)

    def _graph_phase(self, phase, phase_real_img, phase_real_c, phase_gen_z, phase_gen_c):
        st = self._graphs.get(phase.name)
        if st is None:
            st = dnnlib.EasyDict()
            st.inputs = [[t.clone() for t in lst] for lst in (phase_real_img, phase_real_c, phase_gen_z, phase_gen_c)]
            st.params = list(phase.module.parameters())
            phase.opt.zero_grad(set_to_none=True)
            torch.cuda.synchronize(self.device)
            st.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(st.graph):
                phase.module.requires_grad_(True)
                self._accumulate(phase, *st.inputs, arm=False)
                phase.module.requires_grad_(False)
            st.grads = [p.grad for p in st.params]      # the graph writes these buffers on every replay
            self._graphs[phase.name] = st
        else:
            for dst, src in zip(st.inputs, (phase_real_img, phase_real_c, phase_gen_z, phase_gen_c)):
                for d, s_ in zip(dst, src):
                    d.copy_(s_)
        for p, g in zip(st.params, st.grads):
            p.grad = g
        st.graph.replay()

    def step(self, phase_real_img, phase_real_c, all_gen_z, all_gen_c):
        """One iteration.  phase_real_img/c: lists of batch_gpu chunks; all_gen_z/c: per phase, lists
        of chunks (the reference's data layout, :317-323)."""
        for phase, phase_gen_z, phase_gen_c in zip(self.phases, all_gen_z, all_gen_c):
            if self.batch_idx % phase.interval != 0:
                continue
            if phase.start_event is not None:
                phase.start_event.record(torch.cuda.current_stream(self.device))
            if self.graphs:
                self._graph_phase(phase, phase_real_img, phase_real_c, phase_gen_z, phase_gen_c)
            else:
                phase.opt.zero_grad(set_to_none=True)
                phase.module.requires_grad_(True)
                self._accumulate(phase, phase_real_img, phase_real_c, phase_gen_z, phase_gen_c, arm=True)
                phase.module.requires_grad_(False)
            with torch.autograd.profiler.record_function(phase.name + '_opt'):
                phase.reducer.finish()
                if self.on_grads is not None:
                    self.on_grads(phase.name, phase.module)
                phase.opt.step()
            if phase.end_event is not None:
                phase.end_event.record(torch.cuda.current_stream(self.device))

        with torch.autograd.profiler.record_function('Gema'):
            ema_nimg = self.ema_kimg * 1000
            if self.ema_rampup is not None:
                ema_nimg = min(ema_nimg, self.cur_nimg * self.ema_rampup)
            ema_beta = 0.5 ** (self.batch_size / max(ema_nimg, 1e-8))
            with torch.no_grad():
                ema_p = list(self.G_ema.parameters())
                cur_p = list(self.G.parameters())
                torch._foreach_lerp_(ema_p, cur_p, 1.0 - ema_beta)   # p.lerp(p_ema, beta) written into p_ema
                for b_ema, b in zip(self.G_ema.buffers(), self.G.buffers()):
                    b_ema.copy_(b)

        self.cur_nimg += self.batch_size
        self.batch_idx += 1

        if self.ada_stats is not None and self.batch_idx % self.ada_interval == 0:
            self.ada_stats.update()
            adjust = np.sign(self.ada_stats['Loss/signs/real'] - self.ada_target) * \
                (self.batch_size * self.ada_interval) / (self.ada_kimg * 1000)
            self.augment_pipe.p.copy_((self.augment_pipe.p + adjust).max(misc.constant(0, device=self.device)))
        return ema_beta
