"""The product's isolated iteration of a config at states nudged by 2^-<k> (config_parity.run_product perturb, the
same signs and order as the oracle's run_oracle nudge), each saved as gpurun_out/pert/summ_<tag>_<dt>_p<k>_s<seed>.npz
for an offline comparison against the float64 answer and the emulated reference at the same states
(tests/golden/make_golden.py emu16p).  Usage: python tools/prod_perturbed.py <tag> <fp16|bf16> <k> <seed> [seed ...]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import config_parity as cp  # noqa: E402
from golden_init import pack  # noqa: E402

tag, dt, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
dev = torch.device('cuda', 0)
out_dir = os.path.join(ROOT, 'gpurun_out', 'pert')
os.makedirs(out_dir, exist_ok=True)
for seed in [int(v) for v in sys.argv[4:]]:
    cfg, inp, tape, _ = cp.load_fixture(np.load(os.path.join(ROOT, 'tests', 'golden', f'train_{tag}_iso.npz')))
    got, _ = cp.run_product(cfg, inp, tape, dev, fp16_dtype=torch.float16 if dt == 'fp16' else torch.bfloat16,
                            aug_p=cfg['aug_p'], isolated=True, perturb=2.0 ** -k, perturb_seed=seed)
    np.savez_compressed(os.path.join(out_dir, f'summ_{tag}_{dt}_p{k}_s{seed}.npz'), **pack(got))
    print(tag, dt, k, seed, 'saved', flush=True)
