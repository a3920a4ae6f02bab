"""Attribute the f32 atomic-mode error of a phase-isolated fixture per tensor (GPU diagnostic).

    python tools/atomic_attr.py [tag] [runs]

Runs train_<tag>_iso.npz in f32 once in deterministic mode and `runs` times with the float atomics, keeping every
phase's full gradient tensors, and prints per phase:
  * each run's two flat measures against float64 (config_parity.compare_flat) and the reference's;
  * the tensors that carry the measures: per tensor its share of the norm-vector error^2 and of the flat error^2
    (numel x mean sampled-entry error^2), in the worst atomic run and in the det run;
  * the tensors that move between runs: full-tensor relative L2 of each atomic run against the det run.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import config_parity as cp  # noqa: E402
from golden_util import load  # noqa: E402

PH = ['Gmain', 'Greg', 'Dmain', 'Dreg']


def run(tag, det, full):
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}_iso.npz'))
    orig = cp.summarize

    def keep(named, prefix):
        full[prefix] = {n: t.detach().double().clone() for n, t in named.items()}
        return orig(named, prefix)
    cp.summarize = keep
    try:
        got, _ = cp.run_product(cfg, inp, tape, torch.device('cuda', 0), aug_p=cfg['aug_p'], isolated=True,
                                deterministic=det)
    finally:
        cp.summarize = orig
    return got, fix


def shares(got, truth, ph):
    keys = [k for k in cp._keys(truth, (f'grad/{ph}/',)) if k + '/norm' in got]
    nb = np.array([float(truth[k + '/norm']) for k in keys])
    na = np.array([float(got[k + '/norm']) for k in keys])
    tot = float(np.sum(nb ** 2))
    dn = (na - nb) ** 2 / tot
    df = np.array([float(truth[k + '/numel']) * float(np.mean((np.asarray(got[k + '/samples'], np.float64) -
                                                                np.asarray(truth[k + '/samples'], np.float64)) ** 2))
                   for k in keys]) / tot
    return keys, dn, df


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else 'c4'
    nrun = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    res = []
    for i in range(nrun + 1):
        full = {}
        got, fix = run(tag, i == 0, full)
        res.append((got, full))
        truth = {k[4:]: v for k, v in fix.items() if k.startswith('f64/')}
        flat = cp.compare_flat(got, truth, [f'grad/{p}' for p in PH])
        print(f'[{tag} {"det" if i == 0 else f"atomic{i}"}]', {g[5:]: (f'{a:.3g}', f'{b:.3g}') for g, (a, b) in flat.items()},
              flush=True)
    ref = cp.reference_flat(fix, truth, [f'grad/{p}' for p in PH])
    print('[reference spread]', {g[5:]: (f'{a:.3g}', f'{b:.3g}') for g, (a, b) in ref.items()})
    for ph in PH:
        g = f'grad/{ph}'
        flats = [cp.compare_flat(r[0], truth, [g])[g] for r in res]
        worst = 1 + int(np.argmax([f[1] for f in flats[1:]]))
        print(f'\n== {ph}: det {flats[0]}, worst atomic run {worst} {flats[worst]}')
        for lab, idx in (('det', 0), (f'atomic{worst}', worst)):
            keys, dn, df = shares(res[idx][0], truth, ph)
            print(f'  {lab}: norm-vector err^2 {dn.sum():.3g}, flat err^2 {df.sum():.3g}; largest shares:')
            for j in np.argsort(-(dn + df))[:8]:
                k = keys[j]
                print(f'     norm {dn[j] / max(dn.sum(), 1e-300):6.1%} flat {df[j] / max(df.sum(), 1e-300):6.1%}  '
                      f'tensor norm rel err {abs(float(res[idx][0][k + "/norm"]) / float(truth[k + "/norm"]) - 1):.3g}  '
                      f'numel {int(truth[k + "/numel"])}  {k}')
        det_full = res[0][1][g]
        mv = {}
        for r in res[1:]:
            for n, t in r[1][g].items():
                d = det_full[n]
                e = float((t - d).norm() / max(float(d.norm()), 1e-300))
                mv[n] = max(mv.get(n, 0.0), e)
        print('  moved vs det (max over atomic runs, full-tensor rel L2):')
        for n, e in sorted(mv.items(), key=lambda x: -x[1])[:10]:
            print(f'     {e:9.3g}  numel {det_full[n].numel():8d}  {n}')


if __name__ == '__main__':
    main()
