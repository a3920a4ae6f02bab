"""Systematic bias of the f32 convolution forms (GPU): for a few low-resolution layer shapes, the signed shrink
sum((y - y64) * sign(y64)) / sum(|y64|) and the plain relative error of the split-bf16 (S3) and f32-input MFMA
(SG2_F32_EXACT=1) forms against float64.  Random rounding gives a shrink near zero (~1e-9); a directed
rounding in the accumulation shows as a shrink of the size of the error itself.

    python tools/s3_bias.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gan-track_amd'))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from torch_utils.ops import conv2d_gradfix as cg  # noqa: E402

DEV = torch.device('cuda', 0)


def main():
    g = torch.Generator().manual_seed(1)
    for N, C, R, O, k, splitk_note in [(2, 512, 4, 512, 3, 'split-K'), (2, 512, 8, 512, 3, 'split-K'),
                                        (2, 512, 16, 512, 3, ''), (32, 512, 16, 512, 3, ''), (2, 64, 64, 64, 3, '')]:
        x = torch.randn(N, C, R, R, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(O, C, k, k, generator=g)).to(DEV)
        s = (torch.rand(N, C, generator=g) + 0.5).to(DEV)
        y64 = F.conv2d((x.double() * s.double()[:, :, None, None]).cpu(), w.double().cpu(), padding=1)
        res = []
        for exact in ('0', '1'):
            os.environ['SG2_F32_EXACT'] = exact
            cg.presplit = exact == '0'
            y = cg.conv_fused(x, cg._pack_conv(w), O, R, R, k, k, 1, (1, 1), in_scale=s)[0].double().cpu()
            d = y - y64
            shrink = float((d * torch.sign(y64)).sum() / y64.abs().sum())
            res.append(f'{"exact" if exact == "1" else "S3"}: rel {float(d.norm() / y64.norm()):.3g} shrink {shrink:.3g}')
        os.environ.pop('SG2_F32_EXACT')
        print(f'N{N} C{C} {R}^2 -> {O} {splitk_note}: ' + '; '.join(res), flush=True)


if __name__ == '__main__':
    main()
