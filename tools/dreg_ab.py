"""Which kernel path moves the 16-bit Dreg result (GPU): runs the isolated C2 bf16 iteration at the fixture state and
at 2^-12-nudged states with alternative kernel paths switched by environment (the LDS-transposed halo epilogue, the
32x4 halo form for the stride-2 convs, the persistent C=64 kernel instead of the ring, ...), saving each run's
summaries to gpurun_out/dreg_ab/summ_<cfg>_s<seed>.npz for an offline comparison against the float64 answers.
Usage: python tools/dreg_ab.py [seed ...]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import config_parity as cp  # noqa: E402
from golden_init import pack  # noqa: E402

CFGS = {'base': {}, 'halo_lds': {'SG2_HALO_DIRECT': '0'}, 's2_halo': {'SG2_S2G': '0'}, 'c64p': {'SG2_C64_RING': '0'},
        'c32_off': {'SG2_C32_RING': '0'}}
seeds = [int(v) for v in sys.argv[1:]] or [0, 1, 2]
dev = torch.device('cuda', 0)
out_dir = os.path.join(ROOT, 'gpurun_out', 'dreg_ab')
os.makedirs(out_dir, exist_ok=True)
for name, env in CFGS.items():
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    for seed in seeds:
        cfg, inp, tape, _ = cp.load_fixture(np.load(os.path.join(ROOT, 'tests', 'golden', 'train_c2_iso.npz')))
        got, _ = cp.run_product(cfg, inp, tape, dev, fp16_dtype=torch.bfloat16, aug_p=cfg['aug_p'], isolated=True,
                                perturb=2.0 ** -12 if seed else 0.0, perturb_seed=seed)
        np.savez_compressed(os.path.join(out_dir, f'summ_{name}_s{seed}.npz'), **pack(got))
        print(name, seed, 'saved', flush=True)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
