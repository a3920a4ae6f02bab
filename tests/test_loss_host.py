"""StyleGAN2Loss host logic (training/loss.py: phase -> terms, draw order, reported statistics, gains)
on CPU, driven with the oracle's networks and augment pipe: same gradients, statistics and pl_mean as the
oracle's restatement of SG3/training/loss.py:64-139 for every phase and for the degenerate settings
(pl_weight = 0, r1_gamma = 0, the 'both' phases)."""

import numpy as np
import pytest
import torch

from rngtape import Tape
from oracle import sg2_oracle as O
from training import loss as loss_mod


def _nets():
    torch.manual_seed(0)
    G = O.Generator(z_dim=16, c_dim=2, w_dim=16, img_resolution=16, img_channels=1, channel_base=64, channel_max=8,
                    mapping_kwargs=dict(num_layers=2), fused_modconv_default='inference_only').train().requires_grad_(False)
    D = O.Discriminator(c_dim=2, img_resolution=16, img_channels=1, channel_base=64, channel_max=8,
                        epilogue_kwargs=dict(mbstd_group_size=2)).train().requires_grad_(False)
    aug = O.AugmentPipe(xflip=1, xint=1, scale=1, rotate=1, aniso=1, xfrac=1)
    aug.p.fill_(0.5)
    return G, D, aug


def _run(which, phase, pl_weight, r1_gamma, tape):
    G, D, aug = _nets()
    stats = []
    rep = lambda n, v: stats.append((n, torch.as_tensor(v).detach().clone())) or v  # noqa: E731
    kw = dict(augment_pipe=aug, r1_gamma=r1_gamma, style_mixing_prob=0.9, pl_weight=pl_weight, pl_no_weight_grad=True)
    if which == 'oracle':
        loss = O.StyleGAN2Loss(None, G, D, report=rep, **kw)
    else:
        loss = loss_mod.StyleGAN2Loss(device=torch.device('cpu'), G=G, D=D, **kw)
    g = torch.Generator().manual_seed(3)
    real = torch.rand([4, 1, 16, 16], generator=g) * 2 - 1
    c = torch.nn.functional.one_hot(torch.randint(0, 2, [4], generator=g), 2).float()
    z = torch.randn([4, 16], generator=g)
    mod = G if phase.startswith('G') else D
    mod.requires_grad_(True)
    orig = loss_mod.training_stats.report
    loss_mod.training_stats.report = rep
    try:
        with (tape.record() if not tape.entries else tape.replay()):
            loss.accumulate_gradients(phase, real, c, z, c, gain=3, cur_nimg=0)
    finally:
        loss_mod.training_stats.report = orig
    grads = {n: p.grad.clone() for n, p in mod.named_parameters() if p.grad is not None}
    return grads, stats, float(loss.pl_mean)


@pytest.mark.parametrize('phase,pl_weight,r1_gamma', [('Gmain', 2, 1), ('Greg', 2, 1), ('Gboth', 2, 1), ('Greg', 0, 1),
                                                      ('Gboth', 0, 1), ('Dmain', 2, 1), ('Dreg', 2, 1),
                                                      ('Dboth', 2, 1), ('Dreg', 2, 0), ('Dboth', 2, 0)])
def test_loss_phases_match_oracle(phase, pl_weight, r1_gamma):
    tape = Tape(seed=4)
    go, so, plo = _run('oracle', phase, pl_weight, r1_gamma, tape)
    gp, sp, plp = _run('product', phase, pl_weight, r1_gamma, tape)
    assert tape.pos == len(tape.entries), 'different random-draw sequence'
    assert [n for n, _ in sp] == [n for n, _ in so]
    for (n, a), (_, b) in zip(sp, so):
        assert torch.allclose(a.float(), b.float(), rtol=1e-5, atol=1e-6), n
    assert sorted(gp) == sorted(go)
    for k in go:
        assert torch.allclose(gp[k], go[k], rtol=1e-4, atol=1e-7), k
    assert np.isclose(plp, plo, rtol=1e-6)
    if (phase == 'Greg' and pl_weight == 0) or (phase == 'Dreg' and r1_gamma == 0):
        assert not go and not so
