"""Conditioning of the product's own evaluation (GPU): the phase-isolated fixture run with every parameter, real
image and latent nudged by (1 +- rel) (config_parity._perturb, a few sign seeds), next to the unperturbed run and
the float64 answer -- the product-side twin of the oracle's f64p fixtures.  A tensor that the product moves much
further than the float64 oracle moves under the same nudge points at an incoherence in the product (a quantity
evaluated two ways), not at the problem's conditioning.

    python tools/perturb_spread.py c2 [log2_rel=-20] [seeds=3] [substring ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import config_parity as cp  # noqa: E402
from golden_util import load  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else 'c2'
    rel = 2.0 ** float(sys.argv[2]) if len(sys.argv) > 2 else 2.0 ** -20
    seeds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    subs = sys.argv[4:] or ['noise_strength', 'b256.conv1.bias']
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}_iso.npz'))
    truth = {k[4:]: v for k, v in fix.items() if k.startswith('f64/')}
    cond = {k[5:]: v for k, v in fix.items() if k.startswith('f64p/')}
    dev = torch.device('cuda', 0)
    orig_nets = cp._nets
    runs = []
    for s in range(seeds + 1):
        gen = torch.Generator().manual_seed(1000 + s)

        def nets(*a, **k):
            G, D = orig_nets(*a, **k)
            if s:
                with torch.no_grad():
                    for m in (G, D):
                        for _, p in sorted(m.named_parameters()):
                            p.copy_(cp._perturb(p.double(), rel, gen).to(p.dtype))
            return G, D
        cp._nets = nets
        ip = inp if not s else {k: (cp._perturb(torch.from_numpy(np.asarray(v, np.float64)), rel, gen).numpy()
                                    if k in ('real', 'gen_z', 'z') else v) for k, v in inp.items()}
        try:
            got, _ = cp.run_product(cfg, ip, tape, dev, aug_p=cfg['aug_p'], isolated=True)
        finally:
            cp._nets = orig_nets
        runs.append(got)
    keys = [k for ph in ('Gmain', 'Greg', 'Dmain', 'Dreg') for k in cp._keys(truth, (f'grad/{ph}/',))]
    E = lambda a, b, k: max(cp._tensor_errs(a, b, k))  # noqa: E731
    rows = []
    for k in keys:
        if k + '/norm' not in runs[0]:
            continue
        base = E(runs[0], truth, k)
        spread = max(E(r, runs[0], k) for r in runs[1:])
        c = E(cond, truth, k) if k + '/norm' in cond else float('nan')
        ref = E(fix, truth, k)
        rows.append((spread, base, c, ref, k))
    print(f'{tag}: rel 2^{np.log2(rel):.0f}, {seeds} seeds; columns: product spread under the nudge | product vs f64 '
          f'| oracle f64p vs f64 | reference f32 vs f64')
    for r in sorted(rows, reverse=True)[:25]:
        print(f'  {r[0]:9.3g} | {r[1]:9.3g} | {r[2]:9.3g} | {r[3]:9.3g}  {r[4]}')
    for r in rows:
        if any(s in r[4] for s in subs) and 'Greg' in r[4]:
            print(f'  * {r[0]:9.3g} | {r[1]:9.3g} | {r[2]:9.3g} | {r[3]:9.3g}  {r[4]}')


if __name__ == '__main__':
    main()
