"""Re-judges saved 16-bit product summaries (gpurun_out/summ_<tag>_iso_<dt>_<mode>.npz, written by
tests/test_config_gpu.py::test_16bit_phases) against the fixture's current emulation samples, offline (CPU), with
the test's own rule.  Usage: python tools/rejudge16.py"""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
from golden_init import unpack  # noqa: E402
import config_parity as cp  # noqa: E402

FLOOR = {'fp16': 5e-3, 'bf16': 1e-2}
KEY = {'fp16': 'q16', 'bf16': 'qbf'}
GROUPS = ['grad/Gmain', 'grad/Greg', 'grad/Dmain', 'grad/Dreg']
for tag, dt in [('c1', 'fp16'), ('c1', 'bf16'), ('c2', 'fp16'), ('c2', 'bf16'), ('c4', 'fp16'), ('c5', 'bf16')]:
    fix = unpack(np.load(os.path.join(ROOT, 'tests', 'golden', f'train_{tag}_iso.npz')))
    truth = {k[4:]: v for k, v in fix.items() if k.startswith('f64/')}
    pres = sorted({k.split('/', 1)[0] for k in fix if k.split('/', 1)[0] == KEY[dt] or
                   (k.startswith(KEY[dt] + 'n') and '/' in k)})
    refs = {p: cp.compare_flat({k[len(p) + 1:]: v for k, v in fix.items() if k.startswith(p + '/')}, truth, GROUPS)
            for p in pres}
    for mode in ['det', 'atomic']:
        fn = os.path.join(ROOT, 'gpurun_out', f'summ_{tag}_iso_{dt}_{mode}.npz')
        if not os.path.exists(fn):
            continue
        res = cp.compare_flat(unpack(np.load(fn)), truth, GROUPS)
        out = []
        for g, (en, es) in res.items():
            rn, rs = max(r[g][0] for r in refs.values()), max(r[g][1] for r in refs.values())
            tn, ts = max(FLOOR[dt], 2 * rn), max(FLOOR[dt], 2 * rs)
            out.append(f'{g[5:]} {en / tn:.2f}/{es / ts:.2f}{"!" if en > tn or es > ts else ""}')
        print(f'{tag} {dt} {mode} ({len(pres)} samples): ' + '  '.join(out))
