"""Optimiser step and gradient exchange on the GPU (training/optim.py, training/trainer.py):

  * FlatAdam (one sg2_adam_multi launch) == the reference's phase step -- flat cat, /N, nan_to_num(0, +-1e5),
    torch.optim.Adam (foreach) -- over several steps with changing participation (Gmain / Greg share an
    optimiser; a parameter without a gradient is skipped and keeps its step count);
  * EmaLerp (one sg2_lerp_multi) == p.lerp(p_ema, beta) per tensor (training_loop_mi_multimodal.py:363-364);
  * the HIP-graph exchange path with several (simulated) ranks: bucket fills and all_reduces captured in
    the phase graph from the backward's hooks -- same parameters as the eager hook path and as one flat
    exchange.
"""
import copy

import pytest
import torch

from golden_util import rel_err

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


def _params(seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(512, 512, 3, 3), (512,), (7,), (3, 5000), (1,), (64, 32, 1, 1), (4097,)]
    return [torch.randn(s, generator=g).to(DEV) for s in shapes]


@pytest.mark.parametrize('betas', [(0.0, 0.99), (0.9, 0.999)])
def test_flat_adam_matches_torch(betas):
    from training.optim import FlatAdam
    from training.trainer import GradExchange
    ref = [torch.nn.Parameter(p.clone()) for p in _params()]
    mine = [torch.nn.Parameter(p.clone()) for p in _params()]
    mod = torch.nn.ParameterList(mine)
    lr, eps, N = 0.0025 * 0.8, 1e-8, 2
    topt = torch.optim.Adam(ref, lr=lr, betas=betas, eps=eps, foreach=True)
    fopt = FlatAdam(mine, lr=lr, betas=betas, eps=eps)
    ex = GradExchange(mod, num_gpus=1, bucket_mb=4)
    g = torch.Generator().manual_seed(1)
    for step, part in enumerate([range(7), [0, 2, 3, 5], range(7), [1, 4, 6]]):
        grads = {i: torch.randn(ref[i].shape, generator=g).to(DEV) * N for i in part}
        if step == 0:
            grads[0].view(-1)[:3] = torch.tensor([float('nan'), float('inf'), -float('inf')])
            grads[3].view(-1)[7] = 3e7                    # finite and > 1e5: nan_to_num leaves it
        # reference: zero_grad(set_to_none), grads, flat cat / N / nan_to_num / split, Adam.step
        topt.zero_grad(set_to_none=True)
        ps = [ref[i] for i in sorted(part)]
        flat = torch.cat([grads[i].flatten() for i in sorted(part)]) / N
        torch.nan_to_num(flat, nan=0, posinf=1e5, neginf=-1e5, out=flat)
        for p, gg in zip(ps, flat.split([p.numel() for p in ps])):
            p.grad = gg.reshape(p.shape)
        topt.step()
        fopt.zero_grad(set_to_none=True)
        for i in part:
            mine[i].grad = grads[i].clone()
        got = ex.finish('phase')
        fopt.step_flat(ex.flat, ex.offsets, got, grad_scale=1.0 / N, write_grad=True)
        for i in part:
            assert rel_err(mine[i].grad, ref[i].grad) == 0.0, f'step {step}: sanitised grad {i}'
        for i in range(7):
            e = rel_err(mine[i].detach(), ref[i].detach())
            assert e < 1e-6, f'step {step}: param {i} rel err {e:.3g}'
    assert fopt.steps == [topt.state[p]['step'].item() if p in topt.state else 0 for p in ref]


def test_ema_lerp_matches_reference():
    from training.optim import EmaLerp

    class M(torch.nn.Module):
        def __init__(self, ps):
            super().__init__()
            self.ps = torch.nn.ParameterList([torch.nn.Parameter(p) for p in ps])
            self.register_buffer('w_avg', torch.randn(512))

    G = M(_params(2)).to(DEV)
    E = M(_params(3)).to(DEV)
    ref = copy.deepcopy(E)
    ema = EmaLerp(E, G)
    for beta in [0.3, 0.9576]:      # both branches of torch's lerp formula
        ema(beta)
        with torch.no_grad():
            for pe, p in zip(ref.parameters(), G.parameters()):
                pe.copy_(p.lerp(pe, beta))
        for a, b in zip(E.parameters(), ref.parameters()):
            assert torch.equal(a, b)
        assert torch.equal(E.w_avg, G.w_avg)


class _FakeWork:
    def wait(self):
        pass


def test_graph_exchange_overlap_simulated_ranks(monkeypatch):
    """Two ranks simulated on one GPU: all_reduce(t) -> t *= 2 (the sum of two identical ranks) on the
    stream it is issued on.  Eager hook path, graph path (fills and reductions captured from the hooks)
    and the non-overlapped single exchange must give identical parameters.  Six iterations with both reg
    intervals 2: iteration 4 replays all four phase graphs back to back (_replay_step), with Gmain / Greg and
    Dmain / Dreg each sharing one FlatAdam whose step scalars are staged for both phases before either replays."""
    from training.trainer import Trainer
    from golden_util import load
    from parity_train import build_product, CLARO_AUG
    from training import augment_mi, loss as loss_mod
    monkeypatch.setattr(torch.distributed, 'all_reduce', lambda t, async_op=False: (t.mul_(2), _FakeWork())[1])
    z = load('train_claro.npz')
    res = []
    for mode in ['flat', 'eager', 'graph']:
        cfg, G, D = build_product(z, DEV, fp16=False)
        G_ema = copy.deepcopy(G).eval()
        aug = augment_mi.AugmentPipe(run_dir=None, batch_size=cfg['batch'], **CLARO_AUG).train().requires_grad_(False).to(DEV)
        aug.p.copy_(torch.as_tensor(0.3))
        loss = loss_mod.StyleGAN2Loss(device=DEV, G=G, D=D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9,
                                      pl_weight=2, pl_no_weight_grad=True)
        opt = dict(class_name='torch.optim.Adam', lr=0.0025, betas=[0, 0.99], eps=1e-8)
        tr = Trainer(G, D, G_ema, loss, opt, opt, G_reg_interval=2, D_reg_interval=2, batch_size=cfg['batch'],
                     batch_gpu=cfg['batch'], num_gpus=2, rank=0, device=DEV, overlap=(mode != 'flat'),
                     bucket_mb=0.01)
        assert len(tr.phases[0].exchange.buckets) > 4
        gen = torch.Generator(device=DEV)
        gen.manual_seed(5)
        torch.manual_seed(123)
        for it in range(6):
            if it == 1:
                tr.graphs = mode == 'graph'
            real = torch.rand([cfg['batch'], 1, 32, 32], device=DEV, generator=gen) * 2 - 1
            c = torch.nn.functional.one_hot(torch.randint(0, 2, [cfg['batch']], device=DEV, generator=gen), 2).float()
            gz = torch.randn([4, cfg['batch'], cfg['z_dim']], device=DEV, generator=gen)
            tr.step([real], [c], [[gz[i]] for i in range(4)], [[c] for _ in range(4)])
        torch.cuda.synchronize()
        if mode == 'graph':
            assert tr._graphs['Gmain'].overlapped > 0, 'no bucket was exchanged from inside the captured backward'
        res.append(torch.cat([p.detach().double().flatten() for m in (G, D, G_ema) for p in m.parameters()]))
        if mode == 'flat':
            names = [f'{mn}.{n}' for mn, m in (('G', G), ('D', D), ('G_ema', G_ema)) for n, _ in m.named_parameters()]
            sizes = [p.numel() for m in (G, D, G_ema) for p in m.parameters()]

    def worst(a, b):
        d = [(float((x - y).abs().max()), n) for x, y, n in zip(a.split(sizes), b.split(sizes), names)]
        return sorted(d, reverse=True)[:4]
    assert rel_err(res[1], res[0]) < 1e-6, worst(res[1], res[0])
    assert rel_err(res[2], res[0]) < 1e-5, worst(res[2], res[0])


def test_pack_weight_multi_bitwise():
    """sg2_pack_weight_multi (every pack of a phase in one launch) == the per-call sg2_pack_weight, bitwise, over
    mixed dtypes, transposed views, flips and gains."""
    from torch_utils.ops import conv2d_gradfix as cg
    g = torch.Generator().manual_seed(3)
    ws = [torch.nn.Parameter(torch.randn(s, generator=g).to(DEV)) for s in [(512, 512, 3, 3), (64, 1, 1, 1),
                                                                            (3, 70, 3, 3), (96, 40, 3, 3)]]
    forms = [(ws[0], 0, torch.float16, False, 0.04), (ws[0], 1, torch.bfloat16, True, 1.0), (ws[1], 0, None, False, 2.0),
             (ws[2], 0, torch.float16, True, 0.5), (ws[3].transpose(0, 1), 0, torch.float16, False, 1.0),
             (ws[3], 1, torch.float32, True, 0.25)]
    ref = [cg._pack_raw(w, a, dt, fl, sc) for w, a, dt, fl, sc in forms]
    for (w, a, dt, fl, sc), r in zip(forms, ref):     # the per-call pack itself against torch's expression
        t = (w.detach().flip([2, 3]) if fl else w.detach()) * sc
        assert torch.equal(r, t.permute(a, 2, 3, 1 - a).to(dt or w.dtype).contiguous())
    holder = {}
    for rnd in range(2):                          # first scope records the plan, the second packs up front
        with cg.pack_cache(plan=holder):
            got = [cg._pack(w, a, dt, fl, sc) for w, a, dt, fl, sc in forms]
        assert (holder.get('pack_plan') is not None) and (rnd == 0 or all(
            any(o.data_ptr() == x.data_ptr() for o in holder['pack_plan'].outs) for x in got))
        for a, b in zip(got, ref):
            assert a.dtype == b.dtype and torch.equal(a, b)


@pytest.mark.parametrize('graphs', [False, True], ids=['eager', 'graph'])
def test_prepack_steps_bitwise(graphs):
    """Training steps with the phase-start multi-pack (conv2d_gradfix._PackPlan) == without it, bitwise (fp16
    network, deterministic mode): the packs it makes up front are the packs the phase would make."""
    import sg2hip
    from training.trainer import Trainer
    from golden_util import load
    from parity_train import build_product, CLARO_AUG
    from training import augment_mi, loss as loss_mod
    from torch_utils.ops import conv2d_gradfix as cg
    z = load('train_claro.npz')
    res = []
    for pre in (False, True):
        cg.prepack_enabled = pre
        try:
            cfg, G, D = build_product(z, DEV, fp16=True)
            G_ema = copy.deepcopy(G).eval()
            aug = augment_mi.AugmentPipe(run_dir=None, batch_size=cfg['batch'], **CLARO_AUG).train().requires_grad_(False).to(DEV)
            aug.p.copy_(torch.as_tensor(0.3))
            loss = loss_mod.StyleGAN2Loss(device=DEV, G=G, D=D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9,
                                          pl_weight=2, pl_no_weight_grad=True)
            opt = dict(class_name='torch.optim.Adam', lr=0.0025, betas=[0, 0.99], eps=1e-8)
            tr = Trainer(G, D, G_ema, loss, opt, opt, G_reg_interval=2, D_reg_interval=2, batch_size=cfg['batch'],
                         batch_gpu=cfg['batch'], num_gpus=1, rank=0, device=DEV)
            gen = torch.Generator(device=DEV)
            gen.manual_seed(5)
            torch.manual_seed(123)
            with sg2hip.deterministic(device=DEV):
                for it in range(5):
                    if it == 2:
                        tr.graphs = graphs
                    real = torch.rand([cfg['batch'], 1, 32, 32], device=DEV, generator=gen) * 2 - 1
                    c = torch.nn.functional.one_hot(torch.randint(0, 2, [cfg['batch']], device=DEV, generator=gen), 2).float()
                    gz = torch.randn([4, cfg['batch'], cfg['z_dim']], device=DEV, generator=gen)
                    tr.step([real], [c], [[gz[i]] for i in range(4)], [[c] for _ in range(4)])
                torch.cuda.synchronize()
            if pre:
                assert all(ph.get('pack_plan') is not None for ph in tr.phases), 'a phase recorded no pack plan'
            res.append(torch.cat([p.detach().double().flatten() for m in (G, D, G_ema) for p in m.parameters()]))
        finally:
            cg.prepack_enabled = True
    assert torch.equal(res[0], res[1])
