"""Same-state 16-bit samples for a phase-isolated fixture, from the ORACLE only (test infrastructure; no reference
import -- the float64 answer and the emulated reference's 16-bit evaluation at a nudged state are both oracle
evaluations, as make_golden.py's emu16p step makes them):

    PYTHONPATH=tests/golden:tests:gan-track_amd:. python tests/golden/make_same_state.py <tag> <fp16|bf16> <seed>... [--k 12]
    PYTHONPATH=tests/golden:tests:gan-track_amd:. python tests/golden/make_same_state.py <tag> --merge

Each seed writes $GOLD_CACHE/p<k>_<tag>_{f64,<dt>}_<seed>.npz (make_golden.py gen_emulated16_perturbed's format);
--merge folds every cached sample of <tag> into tests/golden/train_<tag>.npz as 'f64p<k>s<seed>/' and
'q16p<k>s<seed>/' / 'qbfp<k>s<seed>/' (make_golden.py merge_emulated16_perturbed), keeping the fixture's other
samples.  A state whose float64 answer the fixture already holds is not re-evaluated (C2's fp16 samples reuse the
float64 answers made with its bf16 ones)."""
import os
import re
import sys
import glob

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))
CACHE = os.environ.get('GOLD_CACHE', '/tmp/gold')


def gen(tag, dt, seed, k):
    import config_parity as cp
    from golden_init import pack
    os.makedirs(CACHE, exist_ok=True)
    for d in ('f64', dt):
        fn = os.path.join(CACHE, f'p{k}_{tag}_{d}_{seed}.npz')
        if os.path.exists(fn):
            continue
        with np.load(os.path.join(OUT, f'train_{tag}.npz'), allow_pickle=False) as f:
            cfg, inp, tape, fix = cp.load_fixture(f)
        pre = {'f64': 'f64', 'fp16': 'q16', 'bf16': 'qbf'}[d] + f'p{k}s{seed}/'
        if any(kk.startswith(pre) for kk in fix):
            print(tag, d, k, seed, 'already in the fixture', flush=True)
            continue
        out, _ = cp.run_oracle_f64(cfg, inp, tape, cfg.get('aug_p', 0.3), perturb=2.0 ** -k, perturb_seed=int(seed),
                                   isolated=cfg.get('isolated', False),
                                   emu16=None if d == 'f64' else {'fp16': torch.float16, 'bf16': torch.bfloat16}[d])
        tmp = fn + '.tmp.npz'
        np.savez_compressed(tmp, **pack(out))
        os.replace(tmp, fn)
        print(tag, d, k, seed, 'same-state sample written', flush=True)


def merge(tag):
    from golden_init import pack, unpack
    path = os.path.join(OUT, f'train_{tag}.npz')
    with np.load(path, allow_pickle=False) as f:
        z = unpack(f)
    n = 0
    for fn in sorted(glob.glob(os.path.join(CACHE, f'p*_{tag}_*.npz'))):
        m = re.match(r'p(\d+)_' + re.escape(tag) + r'_(f64|fp16|bf16)_(\d+)\.npz$', os.path.basename(fn))
        if not m:
            continue
        pre = {'f64': 'f64', 'fp16': 'q16', 'bf16': 'qbf'}[m.group(2)] + f'p{m.group(1)}s{m.group(3)}'
        z = {kk: v for kk, v in z.items() if not kk.startswith(pre + '/')}      # (a cached sample replaces its own)
        with np.load(fn, allow_pickle=False) as f:
            z.update({f'{pre}/{kk}': v for kk, v in unpack(f).items()})
        n += 1
    tmp = path + '.tmp.npz'
    np.savez_compressed(tmp, **pack(z))
    os.replace(tmp, path)
    print(tag, n, 'same-state samples merged', flush=True)


if __name__ == '__main__':
    a = sys.argv[1:]
    k = 12
    if '--k' in a:
        i = a.index('--k')
        k = int(a[i + 1])
        del a[i:i + 2]
    if '--merge' in a:
        merge(a[0])
    else:
        for s in a[2:]:
            gen(a[0], a[1], s, k)
