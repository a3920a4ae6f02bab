"""Whole-network and whole-iteration parity on the GPU (product vs CPU oracle vs reference goldens)."""
import numpy as np
import pytest
import torch

from golden_util import load, rel_err
from parity_train import build_product, run_train_parity

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


@pytest.mark.parametrize('tag', ['claro', 'pelvis'])
def test_forward_inference(tag):
    z = load(f'train_{tag}.npz')
    cfg, G, D = build_product(z, DEV, fp16=False)
    G.eval()
    zz = torch.from_numpy(z['z']).to(DEV)
    cc = torch.from_numpy(z['c']).to(DEV)
    with torch.no_grad():
        img = G(zz, cc, noise_mode='const')
        assert rel_err(img, z['ema_img_const']) < 1e-4
        assert rel_err(D(img, cc), z['D_logits_ema']) < 1e-4
        assert rel_err(G.mapping(zz, cc, truncation_psi=0.7), z['ws_trunc']) < 1e-5


@pytest.mark.parametrize('tag', ['claro', 'pelvis'])
def test_train_iteration_fp32(tag):
    run_train_parity(f'train_{tag}.npz', fp16=False)


@pytest.mark.parametrize('tag', ['claro'])
def test_train_iteration_fp16(tag):
    run_train_parity(f'train_{tag}.npz', fp16=True)


@pytest.mark.gpu
@pytest.mark.parametrize('fp16', [False, True])
def test_graph_mode_matches_eager(fp16):
    """Trainer graph mode (each phase's forward + backward captured once in a HIP graph and replayed)
    reproduces eager training: same RNG draws (graph-safe generator offsets), same kernels, so the
    parameters after three iterations (one eager, then capture + replays covering all four phases) agree
    to rounding."""
    import copy
    from golden_util import load
    from parity_train import build_product, CLARO_AUG
    from training import augment_mi, loss as loss_mod, trainer as trainer_mod
    z = load('train_claro.npz')
    dev = torch.device('cuda', 0)
    res = []
    for graphs in [False, True]:
        cfg, G, D = build_product(z, dev, fp16)
        G_ema = copy.deepcopy(G).eval()
        aug = augment_mi.AugmentPipe(run_dir=None, batch_size=cfg['batch'], **CLARO_AUG).train().requires_grad_(False).to(dev)
        aug.p.copy_(torch.as_tensor(0.3))
        loss = loss_mod.StyleGAN2Loss(device=dev, G=G, D=D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9,
                                      pl_weight=2, pl_no_weight_grad=True)
        opt = dict(class_name='torch.optim.Adam', lr=0.0025, betas=[0, 0.99], eps=1e-8)
        tr = trainer_mod.Trainer(G, D, G_ema, loss, opt, opt, G_reg_interval=2, D_reg_interval=2,
                                 batch_size=cfg['batch'], batch_gpu=cfg['batch'], num_gpus=1, rank=0, device=dev)
        torch.manual_seed(123)
        gen = torch.Generator(device=dev)
        gen.manual_seed(5)
        for it in range(4):
            if it == 1:
                tr.graphs = graphs
            real = torch.rand([cfg['batch'], cfg['img_channels'], cfg['img_resolution'], cfg['img_resolution']],
                              device=dev, generator=gen) * 2 - 1
            c = torch.nn.functional.one_hot(torch.randint(0, cfg['c_dim'], [cfg['batch']], device=dev, generator=gen),
                                            cfg['c_dim']).float()
            gz = torch.randn([4, cfg['batch'], cfg['z_dim']], device=dev, generator=gen)
            tr.step([real], [c], [[gz[i]] for i in range(4)], [[c] for _ in range(4)])
        torch.cuda.synchronize()
        res.append(torch.cat([p.detach().double().flatten() for m in (G, D, G_ema) for p in m.parameters()]))
    assert rel_err(res[1], res[0]) < (1e-5 if not fp16 else 1e-3)
