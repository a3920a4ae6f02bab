"""toRGB tap diagnostic: second-order gradients with the tap on / off, and off / off (determinism baseline)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import sg2hip  # noqa: E402
from torch_utils.ops import modconv  # noqa: E402
from training import networks_stylegan2 as net  # noqa: E402

DEV = torch.device('cuda', 0)
torch.manual_seed(31)
G = net.Generator(z_dim=32, c_dim=0, w_dim=32, img_resolution=64, img_channels=1, channel_base=2048, channel_max=64,
                  num_fp16_res=4, conv_clamp=256, mapping_kwargs=dict(num_layers=2)).to(DEV)
z = torch.randn(4, 32, device=DEV)
dy = torch.randn(4, 1, 64, 64, device=DEV)


def grads(tap):
    modconv.tap_enabled = tap
    ws = G.mapping(z, None).detach().requires_grad_(True)
    img = G.synthesis(ws, noise_mode='const')
    g, = torch.autograd.grad((img * dy).sum(), [ws], create_graph=True)
    g1 = g.detach().clone()
    gs = torch.autograd.grad(g.square().sum(), [ws] + list(G.synthesis.parameters()), allow_unused=True)
    return g1, gs


with sg2hip.deterministic():
    a1, a = grads(True)
    b1, b = grads(False)
    c1, c = grads(False)
print('first-order g: tap vs off equal', torch.equal(a1, b1), ' off vs off', torch.equal(b1, c1))
names = ['ws'] + [n for n, _ in G.synthesis.named_parameters()]
for i, (u, v, w) in enumerate(zip(a, b, c)):
    if u is None:
        continue
    d1 = float((u - v).abs().max()) / max(1e-30, float(v.abs().max()))
    d2 = float((v - w).abs().max()) / max(1e-30, float(v.abs().max()))
    if d1 > 0 or d2 > 0:
        print(f'{names[i]:45s} tap-vs-off {d1:.3g}  off-vs-off {d2:.3g}')
