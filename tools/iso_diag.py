"""Phase-isolated parity diagnostics (GPU): run a train_<tag>_iso.npz fixture through the product under several
switches and list, per phase, the tensors furthest from the float64 answer next to the reference's own f32 error.

    python tools/iso_diag.py c2 [f32|fp16|bf16] [variants...]
variants: base (deterministic), nodet, novjp (modconv.fused_vjp off), nofuse (modconv.enabled off: the composed
layer), noring (SG2_C64_RING=0)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')):
    sys.path.insert(0, p)

import torch  # noqa: E402

import config_parity as cp  # noqa: E402
from golden_util import load  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else 'c2'
    dt = sys.argv[2] if len(sys.argv) > 2 else 'f32'
    variants = sys.argv[3:] or ['base', 'novjp', 'nofuse']
    fdt = {'f32': None, 'fp16': torch.float16, 'bf16': torch.bfloat16}[dt]
    from torch_utils.ops import modconv
    dev = torch.device('cuda', 0)
    for v in variants:
        modconv.fused_vjp = v != 'novjp'
        modconv.enabled = v != 'nofuse'
        if v == 'noring':
            os.environ['SG2_C64_RING'] = '0'
        else:
            os.environ.pop('SG2_C64_RING', None)
        cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}_iso.npz'))
        got, stats = cp.run_product(cfg, inp, tape, dev, fp16_dtype=fdt, aug_p=cfg['aug_p'], isolated=True,
                                    deterministic=v != 'nodet')
        truth = {k[4:]: x for k, x in fix.items() if k.startswith('f64/')}
        flat = cp.compare_flat(got, truth, ['grad/Gmain', 'grad/Greg', 'grad/Dmain', 'grad/Dreg'])
        print(f'== {tag} {dt} {v}: flat', {g: (round(a, 5), round(b, 5)) for g, (a, b) in flat.items()}, flush=True)
        for ph in ('Gmain', 'Greg', 'Dmain', 'Dreg'):
            rows = []
            for k in cp._keys(truth, (f'grad/{ph}/',)):
                if k + '/norm' not in got:
                    continue
                gn, gs = cp._tensor_errs(got, truth, k)
                rn, rs = cp._tensor_errs(fix, truth, k)
                rows.append((max(gn, gs), gn, gs, rn, rs, k))
            rows.sort(reverse=True)
            for r in rows[:6]:
                print(f'   {ph:5s} {r[0]:9.3g}  norm {r[1]:9.3g} samp {r[2]:9.3g} | ref norm {r[3]:9.3g} samp {r[4]:9.3g}  {r[5]}')
        print('   stats worst', cp.judge_stats_f32(stats, fix, check=False), flush=True)


if __name__ == '__main__':
    main()
