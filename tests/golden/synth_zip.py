"""Synthetic Claro / Pelvis-style datasets in the reference's on-disk format (test infrastructure): a zip of
{split}/{patient}/{patient}_{slice:05d}.pickle, each a dict modality -> HxW float64 array in [0, 255], plus
{split}/dataset.json labels (SG3/training/dataset_mi_multimodal.py:193-285; writer src/data/dataset_tool_mi.py).
Deterministic (numpy RandomState): the reference-side fixture generator (make_shell_golden.py) and the tests
build byte-identical decoded images from the same call."""
import json
import pickle
import zipfile

import numpy as np


def make_zip(path, modalities=('CT',), res=16, patients=3, slices=4, labels=True, quirk=False, scale=255.0, peak=False):
    """quirk: add a validation patient whose directory name contains 'train' -- the reference selects a split's
    files by substring (`self._split in fname`), so these belong to the train split too.  scale: the pixel
    range (the FID real-image path treats a batch whose max() is not 255 differently); peak: pixel (0, 0) of
    every slice is exactly 255 (such batches pass the FID path unchanged)."""
    rs = np.random.RandomState(0)
    names, lab = [], []
    with zipfile.ZipFile(path, 'w') as z:
        for split in ('train', 'val'):
            for p in range(patients):
                for s in range(slices):
                    d = {m: (rs.rand(res, res) * scale).astype(np.float64) for m in modalities}
                    if peak:
                        for v in d.values():
                            v[0, 0] = 255.0
                    rel = f'p{p:03d}/p{p:03d}_{s:05d}.pickle'
                    z.writestr(f'{split}/{rel}', pickle.dumps(d))
                    if split == 'train':
                        names.append(rel)
                        lab.append([rel, p % 2])
            if labels:
                z.writestr(f'{split}/dataset.json', json.dumps({'labels': lab if split == 'train' else []}))
        if quirk:
            for s in range(2):
                d = {m: (rs.rand(res, res) * scale).astype(np.float64) for m in modalities}
                z.writestr(f'val/retrain{s}/retrain{s}_{s:05d}.pickle', pickle.dumps(d))
    return names
