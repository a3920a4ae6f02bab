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
