"""One StyleGAN2-ADA training iteration, data-parallel over ranks (one process per GPU).

This is the hot loop of SG3/training/training_loop_mi_multimodal.py:308-376, factored out so the
training loop (training/training_loop.py), bench.py and the tests drive the same code:

    for phase in [Gmain, Greg(every 4), Dmain, Dreg(every 16)]:           (:326-336)
        zero_grad; module.requires_grad_(True); accumulate over batch_gpu chunks
        flat = cat(grads); all_reduce(flat, SUM); flat /= N; nan_to_num  (:341-350)
        Adam step                                                       (:351)
    G_ema = lerp(G, G_ema, beta)                                         (:358-366)
    every ada_interval: p += sign(E[sign(D(real))] - target) * B*I/(ada_kimg*1000)   (:373-376)

Gradient exchange (`GradExchange`).  Each module owns one persistent flat float32 gradient buffer laid
out in backward order (reverse registration) and cut into ~`bucket_mb` MiB buckets.  A bucket is filled
(one cat) as soon as all its parameters hold their final gradient -- from post-accumulate-grad hooks of
the LAST micro-batch's backward -- and, with several ranks, all-reduced asynchronously (RCCL over xGMI,
on RCCL's stream) while the rest of the backward runs.  In HIP-graph mode the same hooks run during
capture, so the fills AND the RCCL all_reduces are captured into the phase graph on a forked stream
branch and joined at its end: a replay overlaps them with the replayed backward (RCCL collectives capture
into hipGraphs on this stack: tools/probe_graph_rccl.py).  The optimiser (training/optim.py FlatAdam,
torch.optim.Adam arithmetic) then reads the flat buffer directly: /N, nan_to_num(0, +-1e5) and Adam are
one launch.  Summation order of the all_reduce differs from the reference's single flat all_reduce only
by fp32 rounding.
"""
import contextlib

import numpy as np
import torch

import dnnlib
from torch_utils import misc
from torch_utils.ops import conv2d_gradfix
from torch_utils import training_stats
from training.optim import FlatAdam, EmaLerp, fused_adam_ok


class GradExchange:
    """Flat, bucketed, backward-overlapped gradient all-reduce of one module's parameters."""

    def __init__(self, module, num_gpus, bucket_mb=32, overlap=True):
        self.params = list(module.parameters())
        self.num_gpus = num_gpus
        self.overlap = overlap and num_gpus > 1
        self.order = list(range(len(self.params)))[::-1]          # backward order
        self.offsets = [0] * len(self.params)
        bucket_elems = max(1, int(bucket_mb * (1 << 20) // 4))
        self.buckets = []                                          # (start, end, [param idx])
        off, cur, start = 0, [], 0
        for i in self.order:
            self.offsets[i] = off
            off += self.params[i].numel()
            cur.append(i)
            if off - start >= bucket_elems:
                self.buckets.append((start, off, cur))
                cur, start = [], off
        if cur:
            self.buckets.append((start, off, cur))
        self.bucket_of = {i: b for b, (_, _, idx) in enumerate(self.buckets) for i in idx}
        self.total = off
        self.flat = None
        self.expect = {}         # phase name -> participating parameter indices (learned from the last run)
        self._zeros = {}
        self._reset()

    def _reset(self):
        self._filled = [False] * len(self.buckets)
        self._works = []
        self._hooks = []
        self._ready = [0] * len(self.buckets)

    def _flat(self, device):
        if self.flat is None or self.flat.device != device:
            self.flat = torch.zeros([self.total], dtype=torch.float32, device=device)
        return self.flat

    def _fill(self, b):
        """Copy bucket b's gradients into its flat range (zeros for a parameter without one)."""
        s, e, idx = self.buckets[b]
        grads = []
        for i in idx:
            g = self.params[i].grad
            if g is None:
                z = self._zeros.get(i)
                if z is None:
                    z = self._zeros[i] = torch.zeros_like(self.params[i])
                g = z
            grads.append(g.reshape(-1))
        flat = self._flat(grads[0].device)
        torch.cat(grads, out=flat[s:e])
        self._filled[b] = True

    def _reduce(self, b):
        if self.num_gpus > 1:
            s, e, _ = self.buckets[b]
            self._works.append(torch.distributed.all_reduce(self.flat[s:e], async_op=True))

    def arm(self, phase, passes=1):
        """Before the last micro-batch: fill and all-reduce each bucket once every participating parameter
        in it has accumulated `passes` gradients (eagerly, or into the graph being captured)."""
        self._reset()
        if not self.overlap:
            return
        part = set(self.expect.get(phase, range(len(self.params))))
        need = [sum(1 for i in idx if i in part) * passes for _, _, idx in self.buckets]

        def hook(p, i):
            b = self.bucket_of[i]
            if p.grad is None or i not in part or self._filled[b]:
                return
            self._ready[b] += 1
            if self._ready[b] == need[b]:
                self._fill(b)
                self._reduce(b)

        self._hooks = [p.register_post_accumulate_grad_hook(lambda p_, i_=i: hook(p_, i_))
                       for i, p in enumerate(self.params) if p.requires_grad]

    def disarm(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def fill_rest(self):
        """Fill every bucket the hooks did not (end of the backward, or of a phase graph)."""
        self.disarm()
        for b in range(len(self.buckets)):
            if not self._filled[b]:
                self._fill(b)

    def close_capture(self):
        """End of a captured phase: fill and reduce the remaining buckets and join every collective back
        into the capture stream, so the graph ends with the exchange complete."""
        self.disarm()
        hooked = sum(self._filled)
        for b in range(len(self.buckets)):
            if not self._filled[b]:
                self._fill(b)
                self._reduce(b)
        for w in self._works:
            w.wait()
        self._reset()
        return hooked

    def finish(self, phase, part=None):
        """Complete the exchange: fill / reduce what is left, wait, point each participating parameter's
        .grad at its range of the flat buffer.  Returns the participating parameter indices (those with a
        gradient; a replayed graph passes the set it captured)."""
        learn = part is None
        if part is None:
            part = [i for i in range(len(self.params)) if self.params[i].grad is not None]
        if not any(self._filled):
            self.fill_rest()
            for b in range(len(self.buckets)):
                self._reduce(b)
        else:
            self.disarm()
            for b in range(len(self.buckets)):
                if not self._filled[b]:
                    self._fill(b)
                    self._reduce(b)
        for w in self._works:
            w.wait()
        self._works = []
        if learn:
            self.expect[phase] = part
        for i in part:
            p = self.params[i]
            p.grad = self.flat[self.offsets[i]:self.offsets[i] + p.numel()].view_as(p)
        self._reset()
        return part


class _HostEvent:
    """Host-clock stand-in for a timing HIP event (exchange diagnostics on a CPU device: the gloo tests)."""

    def record(self, stream=None):
        import time
        self.t = time.perf_counter()

    def elapsed_time(self, end):
        return (end.t - self.t) * 1e3


class Trainer:
    def __init__(self, G, D, G_ema, loss, G_opt_kwargs, D_opt_kwargs, G_reg_interval=4, D_reg_interval=16,
                 batch_size=32, batch_gpu=32, num_gpus=1, rank=0, device=None, ema_kimg=10, ema_rampup=0.05,
                 augment_pipe=None, ada_target=None, ada_interval=4, ada_kimg=500, bucket_mb=32, overlap=True,
                 phase_timing=False, graphs=False, deterministic=True):
        self.G, self.D, self.G_ema, self.loss = G, D, G_ema, loss
        # the library's fixed-order reductions (sg2hip.deterministic) for every phase's forward and backward: the
        # iteration is bitwise reproducible run to run, and measured faster than the float-atomic reductions on the
        # bench workload (747 vs 740 img/s, profiles/r06e_*); False selects the float atomics (an A/B mode)
        self.deterministic = deterministic
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
            exchange = GradExchange(module, num_gpus, bucket_mb=bucket_mb, overlap=overlap)
            kw = dnnlib.EasyDict(opt_kwargs)
            if reg_interval is not None:          # lazy regularisation (:248-255)
                ratio = reg_interval / (reg_interval + 1)
                kw.lr = kw.lr * ratio
                kw.betas = [b ** ratio for b in kw.betas]
            if fused_adam_ok(kw, device):
                opt = FlatAdam(module.parameters(), **{k: v for k, v in kw.items() if k != 'class_name'})
            else:
                opt = dnnlib.util.construct_class_by_name(module.parameters(), **kw)
            if reg_interval is None:
                self.phases.append(dnnlib.EasyDict(name=name + 'both', module=module, opt=opt, interval=1,
                                                   exchange=exchange))
            else:
                self.phases.append(dnnlib.EasyDict(name=name + 'main', module=module, opt=opt, interval=1,
                                                   exchange=exchange))
                self.phases.append(dnnlib.EasyDict(name=name + 'reg', module=module, opt=opt,
                                                   interval=reg_interval, exchange=exchange))
        for ph in self.phases:
            ph.start_event = ph.end_event = None
            if phase_timing and device is not None and device.type == 'cuda':
                ph.start_event = torch.cuda.Event(enable_timing=True)
                ph.end_event = torch.cuda.Event(enable_timing=True)
        self.ema = EmaLerp(G_ema, G) if isinstance(self.phases[0].opt, FlatAdam) else None
        self.cur_nimg = 0
        self.batch_idx = 0
        self.on_grads = None   # optional callback(phase_name, module) after the gradient exchange
        # exchange diagnostics (bench.py at N > 1, eager steps only): per phase a list of (start, backward issued,
        # exchange complete) HIP events on the compute stream -- complete - issued is the part of the bucketed
        # all-reduce the backward did not hide
        self.exchange_timing = None
        # HIP-graph mode: each phase's forward + backward (all micro-batches) and its bucket fills are
        # captured once and replayed (with the gradient exchange); the optimiser, EMA and ADA stay eager.  Capture the
        # first time a phase runs in graph mode -- run at least one eager step first so every lazily created
        # state (kernel attributes, statistics rows, cached constants, participation sets) exists.
        self.graphs = graphs
        self._graphs = {}
        self._static_real = None       # graph-mode static copy of the real batch, shared by the phase graphs
        self._real_staged = None       # the step (self._serial) whose real batch is in it
        self._serial = 0               # step() calls so far (batch_idx may be reset by the caller)

    graph_opt = True     # the FlatAdam launch joins the phase graph (False: stepped eagerly after the replay)

    @staticmethod
    def _passes(name):
        return 2 if name in ('Dmain', 'Dboth') else 1    # D phases backward once for fakes, once for reals

    def _accumulate(self, phase, phase_real_img, phase_real_c, phase_gen_z, phase_gen_c):
        chunks = list(zip(phase_real_img, phase_real_c, phase_gen_z, phase_gen_c))
        # the phase's weights are fixed until its optimizer step: every pack made once, all in one launch at the
        # phase start from the second run on (the plan recorded by the first, kept on the phase)
        with conv2d_gradfix.pack_cache(plan=phase), self._arith():
            for ci, (real_img, real_c, gen_z, gen_c) in enumerate(chunks):
                if ci == len(chunks) - 1:
                    passes = self.loss.backward_passes(phase.name, gen_z.shape[0] + real_img.shape[0]) \
                        if hasattr(self.loss, 'backward_passes') else self._passes(phase.name)
                    phase.exchange.arm(phase.name, passes)
                self.loss.accumulate_gradients(phase=phase.name, real_img=real_img, real_c=real_c, gen_z=gen_z,
                                               gen_c=gen_c, gain=phase.interval, cur_nimg=self.cur_nimg)

    def _arith(self):
        """The reduction mode of the phase passes: deterministic (default) or float-atomic (sg2hip.deterministic)."""
        if self.device is None or self.device.type != 'cuda':
            return contextlib.nullcontext()
        import sg2hip
        return sg2hip.deterministic(self.deterministic, device=self.device)

    def _graph_phase(self, phase, phase_real_img, phase_real_c, phase_gen_z, phase_gen_c):
        """Replay the phase's graph (capturing it the first time): forward + backward of every micro-batch,
        the bucket fills, (several ranks) the overlapped all_reduces and, with FlatAdam, the optimiser
        launch.  Returns (participating parameter indices, whether the optimiser step was in the graph)."""
        st = self._graphs.get(phase.name)
        ex = phase.exchange
        fused_opt = isinstance(phase.opt, FlatAdam)
        if st is None:
            st = dnnlib.EasyDict()
            # the real batch is the same for every phase of a step: one static copy shared by the phase graphs
            if self._static_real is None:
                self._static_real = [[t.clone() for t in lst] for lst in (phase_real_img, phase_real_c)]
                self._real_staged = self._serial
            st.inputs = self._static_real + [[t.clone() for t in lst] for lst in (phase_gen_z, phase_gen_c)]
            self._stage(st, phase, (phase_real_img, phase_real_c), (phase_gen_z, phase_gen_c))
            phase.opt.zero_grad(set_to_none=True)
            flat = ex._flat(self.device)
            # the optimiser launch joins the graph when the participation set learned by the eager warm-up
            # step is known: its tables and step-scalar buffer are built here, outside the capture
            part0 = ex.expect.get(phase.name)
            # (a phase without gradients -- e.g. Greg with pl_weight 0 -- has no Adam launch to capture)
            st.opt_in_graph = fused_opt and bool(part0) and self.graph_opt
            if st.opt_in_graph:
                phase.opt._table(flat, ex.offsets, part0, phase.name)
                if phase.opt.exp_avg is None:
                    phase.opt.exp_avg = torch.zeros_like(flat)
                    phase.opt.exp_avg_sq = torch.zeros_like(flat)
            want_opt = st.opt_in_graph

            def body():
                phase.module.requires_grad_(True)
                self._accumulate(phase, *st.inputs)
                st.part = [i for i, p in enumerate(ex.params) if p.grad is not None]
                st.overlapped = ex.close_capture()
                phase.module.requires_grad_(False)
                st.opt_in_graph = want_opt and st.part == part0
                if st.opt_in_graph:
                    phase.opt.launch(flat, st.part, grad_scale=1.0 / self.num_gpus,
                                     write_grad=self.on_grads is not None, tag=phase.name)
            st.graph = self._capture(body, phase)
            self._graphs[phase.name] = st
            training_stats.mark_captured()
            st.views = False
        else:
            self._stage(st, phase, (phase_real_img, phase_real_c), (phase_gen_z, phase_gen_c))
        if st.opt_in_graph:
            phase.opt.prepare(ex.flat, ex.offsets, st.part, phase.name)   # the step scalars, ordered before the replay
        st.graph.replay()
        ex._filled = [True] * len(ex.buckets)     # filled and reduced inside the graph
        if st.opt_in_graph and st.views:
            ex._reset()
        else:
            # point each .grad at its range of the flat buffer (once: a replay does not touch the attributes)
            ex.finish(phase.name, st.part)
            st.views = True
        return st.part, st.opt_in_graph

    graph_impl = None    # tests: a host stand-in for the capture, graph_impl(body, phase) -> object with replay()

    def _capture(self, body, phase):
        """Capture body() -- the phase's forward / backward, bucket fills, all_reduces (several ranks) and
        optimiser launch -- into a HIP graph and return it.  `graph_impl` replaces the capture on hosts without
        a GPU (tests/test_dist_gloo.py drives the phase-graph bookkeeping at world size 2 with it)."""
        if self.graph_impl is not None:
            return self.graph_impl(body, phase)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body()
        return g

    def _stage(self, st, phase, real, gen):
        """Copy a phase's inputs into its graph's static buffers (the shared real batch only once a step)."""
        if self._real_staged != self._serial:
            for dst, src in zip(self._static_real, real):
                for d, s_ in zip(dst, src):
                    d.copy_(s_)
            self._real_staged = self._serial
        for dst, src in zip(st.inputs[2:], gen):
            for d, s_ in zip(dst, src):
                d.copy_(s_)

    def _replay_step(self, active, phase_real_img, phase_real_c):
        """Graph mode with every active phase captured, its Adam launch inside its graph and its .grad views
        in place: stage all inputs and step scalars first, then replay the phase graphs back to back.  ROCm's
        graph launch returns when the graph's last kernels are queued, so host work between two replays is
        GPU idle time; here there is none (the step scalars of a phase live in a buffer of their own, keyed
        by phase and participation set, so staging every phase first cannot overwrite another's)."""
        for phase, gz, gc in active:
            st = self._graphs[phase.name]
            self._stage(st, phase, (phase_real_img, phase_real_c), (gz, gc))
            phase.opt.prepare(phase.exchange.flat, phase.exchange.offsets, st.part, phase.name)
        for phase, _, _ in active:
            st = self._graphs[phase.name]
            if phase.start_event is not None:
                phase.start_event.record(torch.cuda.current_stream(self.device))
            st.graph.replay()
            if phase.end_event is not None:
                phase.end_event.record(torch.cuda.current_stream(self.device))
        for phase, _, _ in active:
            phase.exchange._reset()

    def step(self, phase_real_img, phase_real_c, all_gen_z, all_gen_c):
        """One iteration.  phase_real_img/c: lists of batch_gpu chunks; all_gen_z/c: per phase, lists
        of chunks (the reference's data layout, :317-323)."""
        self._serial += 1
        if self.graphs and getattr(self.loss, 'blur_fade_kimg', 0) > 0 and getattr(self.loss, 'blur_init_sigma', 0) > 0:
            # the D-input blur fades with cur_nimg, a host float a captured phase would freeze: stay eager
            self.graphs = False
        active = [(ph, gz, gc) for ph, gz, gc in zip(self.phases, all_gen_z, all_gen_c)
                  if self.batch_idx % ph.interval == 0]
        ready = self.graphs and self.on_grads is None and all(
            ph.name in self._graphs and self._graphs[ph.name].opt_in_graph and self._graphs[ph.name].views
            for ph, _, _ in active)
        if ready:
            self._replay_step(active, phase_real_img, phase_real_c)
            active = []
        for phase, phase_gen_z, phase_gen_c in active:
            if phase.start_event is not None:
                phase.start_event.record(torch.cuda.current_stream(self.device))
            part, stepped, finished = None, False, False
            if self.graphs:
                part, stepped = self._graph_phase(phase, phase_real_img, phase_real_c, phase_gen_z, phase_gen_c)
            else:
                evs = None
                if self.exchange_timing is not None:
                    cuda = self.device is not None and self.device.type == 'cuda'
                    evs = [torch.cuda.Event(enable_timing=True) if cuda else _HostEvent() for _ in range(3)]
                    stream = torch.cuda.current_stream(self.device) if cuda else None
                    evs[0].record(stream)
                phase.opt.zero_grad(set_to_none=True)
                phase.module.requires_grad_(True)
                self._accumulate(phase, phase_real_img, phase_real_c, phase_gen_z, phase_gen_c)
                phase.module.requires_grad_(False)
                if evs is not None:
                    evs[1].record(stream)
                    part, finished = phase.exchange.finish(phase.name), True
                    evs[2].record(stream)
                    self.exchange_timing.setdefault(phase.name, []).append(evs)
            with torch.autograd.profiler.record_function(phase.name + '_opt'):
                ex = phase.exchange
                if stepped:
                    # exchange and Adam ran inside the replayed graph (the /N, nan_to_num and write-back of
                    # the scaled gradient included), so there is nothing left to launch for this phase
                    if self.on_grads is not None:
                        self.on_grads(phase.name, phase.module)
                    if phase.end_event is not None:
                        phase.end_event.record(torch.cuda.current_stream(self.device))
                    continue
                part = ex.finish(phase.name, part) if not (self.graphs or finished) else part
                if isinstance(phase.opt, FlatAdam):
                    phase.opt.step_flat(ex.flat, ex.offsets, part, grad_scale=1.0 / self.num_gpus,
                                        write_grad=self.on_grads is not None, tag=phase.name)
                else:
                    flat = ex.flat
                    if self.num_gpus > 1:
                        flat /= self.num_gpus
                    misc.nan_to_num(flat, nan=0, posinf=1e5, neginf=-1e5, out=flat)
                if self.on_grads is not None:
                    self.on_grads(phase.name, phase.module)
                if not isinstance(phase.opt, FlatAdam):
                    phase.opt.step()
            if phase.end_event is not None:
                phase.end_event.record(torch.cuda.current_stream(self.device))

        with torch.autograd.profiler.record_function('Gema'):
            ema_nimg = self.ema_kimg * 1000
            if self.ema_rampup is not None:
                ema_nimg = min(ema_nimg, self.cur_nimg * self.ema_rampup)
            ema_beta = 0.5 ** (self.batch_size / max(ema_nimg, 1e-8))
            with torch.no_grad():
                if self.ema is not None:
                    self.ema(ema_beta)
                else:
                    for p_ema, p in zip(self.G_ema.parameters(), self.G.parameters()):
                        p_ema.copy_(p.lerp(p_ema, ema_beta))
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
