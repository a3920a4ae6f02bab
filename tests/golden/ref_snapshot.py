"""Write a network snapshot with the REFERENCE's own code (test infrastructure; run in a subprocess by
tests/test_trainer_shell.py::test_snapshot_from_reference, only where /root/reference exists -- the pickle embeds
the reference's source text, so it is never committed).

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference/src/models/stylegan3:tests/golden \\
        python tests/golden/ref_snapshot.py <out.pkl> <out.npz>

As the reference's training loop does (SG3/training/training_loop_mi_multimodal.py:420-434): dict(G, D, G_ema,
augment_pipe, training_set_kwargs), every module deep-copied, eval(), requires_grad_(False), on the CPU, pickled
with persistent classes (torch_utils/persistence.py:35-130).  <out.npz> holds every parameter and buffer and the
constructor arguments, for the comparison."""
import copy
import pickle
import sys
import types

import numpy as np

sys.modules['openpyxl'] = types.ModuleType('openpyxl')
import torch  # noqa: E402

import dnnlib  # noqa: E402  (the reference's)
from training import networks_stylegan2 as net, augment_mi  # noqa: E402
from golden_init import init_state  # noqa: E402


def main(pkl_path, npz_path):
    torch.manual_seed(0)
    G = net.Generator(z_dim=32, c_dim=2, w_dim=32, img_resolution=32, img_channels=1, channel_base=256,
                      channel_max=32, num_fp16_res=4, conv_clamp=256, fused_modconv_default='inference_only',
                      mapping_kwargs=dict(num_layers=8))
    D = net.Discriminator(c_dim=2, img_resolution=32, img_channels=1, channel_base=256, channel_max=32, num_fp16_res=4,
                          conv_clamp=256, epilogue_kwargs=dict(mbstd_group_size=4))
    init_state(G, seed=1)
    init_state(D, seed=2)
    G_ema = copy.deepcopy(G)
    with torch.no_grad():
        for p in G_ema.parameters():
            p.mul_(0.5)
    A = augment_mi.AugmentPipe(run_dir=None, batch_size=4, xflip=1, xint=1, scale=1, rotate=1, aniso=1, xfrac=1,
                               xint_max=0.05, rotate_max=3 / 360, xfrac_std=0.05, scale_std=0.05, aniso_std=0.05)
    A.p.fill_(0.375)
    data = dict(G=G, D=D, G_ema=G_ema, augment_pipe=A,
                training_set_kwargs=dict(dnnlib.EasyDict(class_name='training.dataset_mi_multimodal.CustomImageFolderDataset',
                                                         path='claro.zip', split='train', modalities=['CT'])))
    for key, value in data.items():
        if isinstance(value, torch.nn.Module):
            data[key] = copy.deepcopy(value).eval().requires_grad_(False).cpu()
    with open(pkl_path, 'wb') as f:
        pickle.dump(data, f)
    out = {}
    for key in ('G', 'D', 'G_ema', 'augment_pipe'):
        for n, t in list(data[key].named_parameters()) + list(data[key].named_buffers()):
            out[f'{key}/{n}'] = t.detach().numpy()
        out[f'{key}/init_kwargs'] = np.array(repr(dict(data[key].init_kwargs)))
    np.savez(npz_path, **out)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
