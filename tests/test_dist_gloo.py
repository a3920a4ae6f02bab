"""Data-parallel gradient exchange (training/trainer.py GradExchange) with world_size 2 on CPU/gloo.

The product's trainer is driven with the CPU oracle networks (the trainer is device-agnostic host
logic; the HIP ops need a GPU).  Checked: bucketed, backward-overlapped all_reduce gives exactly
mean-over-ranks of each rank's local gradients (reference semantics training_loop:341-350), and
replicas stay bit-identical after the optimizer step (misc.check_ddp_consistency)."""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, paths, result_q):
    import sys
    sys.path[:0] = paths
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.set_num_threads(1)
    try:
        from oracle import sg2_oracle as O
        from training.trainer import Trainer
        from torch_utils import misc
        torch.manual_seed(0)
        G = O.Generator(z_dim=16, c_dim=0, w_dim=16, img_resolution=16, img_channels=1, channel_base=64,
                        channel_max=8, mapping_kwargs=dict(num_layers=2),
                        fused_modconv_default='inference_only').train().requires_grad_(False)
        D = O.Discriminator(c_dim=0, img_resolution=16, img_channels=1, channel_base=64, channel_max=8,
                            epilogue_kwargs=dict(mbstd_group_size=2)).train().requires_grad_(False)
        init = (copy.deepcopy(G.state_dict()), copy.deepcopy(D.state_dict()))
        opt = dict(class_name='torch.optim.Adam', lr=0.0025, betas=[0, 0.99], eps=1e-8)
        B = 4
        g = torch.Generator().manual_seed(10 + rank)
        real = torch.rand([B, 1, 16, 16], generator=g) * 2 - 1
        zs = torch.randn([4, B, 16], generator=g)
        c = torch.zeros([4, B, 0])

        def run(num_gpus, overlap=True, bucket_mb=0.0005, timing=False):
            G.load_state_dict(init[0])
            D.load_state_dict(init[1])
            G_ema = copy.deepcopy(G).eval()
            loss = O.StyleGAN2Loss(None, G, D, r1_gamma=0.5, style_mixing_prob=0.5, pl_weight=2)
            tr = Trainer(G, D, G_ema, loss, opt, dict(opt), batch_size=B * world, batch_gpu=B // 2, num_gpus=num_gpus,
                         rank=rank, device=torch.device('cpu'), bucket_mb=bucket_mb, overlap=overlap)
            grads = {}

            def cb(name, module):
                for n, p in module.named_parameters():
                    if p.grad is not None:
                        grads[f'{name}/{n}'] = p.grad.detach().clone()

            tr.on_grads = cb
            if timing:
                tr.exchange_timing = {}     # bench.py's N > 1 exchange diagnostics (events around finish())
            torch.manual_seed(1234 + rank)
            chunks = lambda t: list(t.split(B // 2))  # noqa: E731
            tr.step(chunks(real), chunks(torch.zeros([B, 0])), [chunks(zs[i]) for i in range(4)],
                    [chunks(c[i]) for i in range(4)])
            return grads, tr

        local, _ = run(1)
        plain, _ = run(world, overlap=False, bucket_mb=1024)   # the reference's single flat all_reduce
        reduced, tr = run(world)                               # bucketed, overlapped with backward
        worst = 0.0
        # Gmain is the first phase: its reduced gradient must be the mean of the ranks' local ones.
        for k in sorted(local):
            if not k.startswith('Gmain/'):
                continue
            others = [torch.zeros_like(local[k]) for _ in range(world)]
            dist.all_gather(others, local[k])
            mean = sum(others) / world
            worst = max(worst, float((reduced[k] - mean).abs().max() / (mean.abs().max() + 1e-12)))
        # Every phase: bucketed/overlapped exchange == one flat all_reduce.
        assert sorted(plain) == sorted(reduced)
        for k in plain:
            worst = max(worst, float((reduced[k] - plain[k]).abs().max() / (plain[k].abs().max() + 1e-12)))
        misc.check_ddp_consistency(G, ignore_regex=r'.*\.[^.]+_(avg|ema)')
        misc.check_ddp_consistency(D)
        nbuckets = len(tr.phases[0].exchange.buckets)
        # with the exchange diagnostics on: the same gradients (finish() runs once per phase, nothing reduced
        # twice) and one (start, issued, complete) record per phase
        timed, trt = run(world, timing=True)
        assert sorted(timed) == sorted(plain)
        for k in plain:
            worst = max(worst, float((timed[k] - plain[k]).abs().max() / (plain[k].abs().max() + 1e-12)))
        assert sorted(trt.exchange_timing) == sorted(ph.name for ph in trt.phases), sorted(trt.exchange_timing)
        assert all(len(v) == 1 and v[0][1].elapsed_time(v[0][2]) >= 0 for v in trt.exchange_timing.values())
        result_q.put((rank, worst, len(local), nbuckets))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_gradient_exchange_gloo():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = [os.path.join(root, 'gan-track_amd'), root]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, paths, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted(q.get(timeout=5) for _ in range(2))
    for rank, worst, n, nb in res:
        assert n > 20
        assert nb > 3, 'test should exercise several buckets'
        assert worst < 1e-6, (rank, worst)


class _HostGraph:
    """CPU stand-in for a captured phase graph (Trainer.graph_impl).  A capture records without executing: the
    stand-in runs the phase body once with the random state forked (a capture consumes no draws of the step), then
    restores the state the body updates in place (the path-length mean) and drops the gradients it made.  A replay clears the module's gradients -- a real replay rewrites the gradient
    buffers its capture allocated, instead of accumulating into the flat views finish() installed -- and runs
    the body again, with its bucket fills and gloo all_reduces, as the replayed graph re-issues the captured
    fills and collectives."""
    captures = 0
    replays = 0

    def __init__(self, body, phase, loss):
        self.body, self.phase = body, phase
        _HostGraph.captures += 1
        pl_mean = loss.pl_mean.clone()
        with torch.random.fork_rng(devices=[]):
            body()
        loss.pl_mean.copy_(pl_mean)
        phase.opt.zero_grad(set_to_none=True)

    def replay(self):
        _HostGraph.replays += 1
        self.phase.opt.zero_grad(set_to_none=True)
        self.body()


def _graph_worker(rank, world, port, paths, result_q):
    """Eager steps vs the phase-graph path (Trainer._graph_phase: static input staging, participation sets,
    capture-time exchange close, per-replay .grad views, /N) at world size 2: same parameters after every step."""
    import sys
    sys.path[:0] = paths
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.set_num_threads(1)
    try:
        from oracle import sg2_oracle as O
        from training.trainer import Trainer
        from torch_utils import misc
        torch.manual_seed(0)
        G = O.Generator(z_dim=16, c_dim=0, w_dim=16, img_resolution=16, img_channels=1, channel_base=64,
                        channel_max=8, mapping_kwargs=dict(num_layers=2),
                        fused_modconv_default='inference_only').train().requires_grad_(False)
        D = O.Discriminator(c_dim=0, img_resolution=16, img_channels=1, channel_base=64, channel_max=8,
                            epilogue_kwargs=dict(mbstd_group_size=2)).train().requires_grad_(False)
        init = (copy.deepcopy(G.state_dict()), copy.deepcopy(D.state_dict()))
        opt = dict(class_name='torch.optim.Adam', lr=0.0025, betas=[0, 0.99], eps=1e-8)
        B, steps = 4, 5
        g = torch.Generator().manual_seed(20 + rank)
        reals = torch.rand([steps, B, 1, 16, 16], generator=g) * 2 - 1
        zs = torch.randn([steps, 4, B, 16], generator=g)
        c = torch.zeros([4, B, 0])
        chunks = lambda t: list(t.split(B // 2))  # noqa: E731

        def run(graphs):
            G.load_state_dict(init[0])
            D.load_state_dict(init[1])
            G_ema = copy.deepcopy(G).eval()
            loss = O.StyleGAN2Loss(None, G, D, r1_gamma=0.5, style_mixing_prob=0.5, pl_weight=2)
            tr = Trainer(G, D, G_ema, loss, opt, dict(opt), G_reg_interval=2, D_reg_interval=2, batch_size=B * world,
                         batch_gpu=B // 2, num_gpus=world, rank=rank, device=torch.device('cpu'), bucket_mb=0.0005)
            tr.graph_impl = lambda body, phase: _HostGraph(body, phase, loss)
            snaps = []
            for s in range(steps):
                tr.graphs = graphs and s >= 1    # one eager step first, as bench.py warms up
                torch.manual_seed(777 + 13 * s + rank)
                tr.step(chunks(reals[s]), chunks(torch.zeros([B, 0])), [chunks(zs[s, i]) for i in range(4)],
                        [chunks(c[i]) for i in range(4)])
                snaps.append([p.detach().clone() for m in (G, D, G_ema) for p in m.parameters()])
            return snaps, tr

        eager, _ = run(False)
        graph, tr = run(True)
        worst = 0.0
        for a, b in zip(eager, graph):
            for x, y in zip(a, b):
                worst = max(worst, float((x - y).abs().max() / (x.abs().max() + 1e-12)))
        misc.check_ddp_consistency(G, ignore_regex=r'.*\.[^.]+_(avg|ema)')
        misc.check_ddp_consistency(D)
        result_q.put((rank, worst, sorted(tr._graphs), _HostGraph.captures, _HostGraph.replays))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_graph_phase_exchange_gloo():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = [os.path.join(root, 'gan-track_amd'), root]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_graph_worker, args=(r, 2, port, paths, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted(q.get(timeout=5) for _ in range(2))
    for rank, worst, captured, ncap, nrep in res:
        assert captured == ['Dmain', 'Dreg', 'Gmain', 'Greg'], captured
        assert ncap == 4 and nrep >= 8, (ncap, nrep)
        assert worst == 0.0, (rank, worst)
