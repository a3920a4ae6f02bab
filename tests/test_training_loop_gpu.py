"""End-to-end run of the training loop on the GPU (training/training_loop_mi_multimodal.py through
train_mi_multimodal.build_config / launch_training): a tiny Claro-like zip, two ticks with ADA, snapshot
pickles, image grids, stats.jsonl with the reference's statistic names, FID per modality with a supplied
detector (a fixed random projection -- the Inception pickle cannot be fetched offline), then a resume from
the last snapshot (the loaded networks equal the saved ones)."""
import json
import os
import pickle
import zipfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _ProjDetector(torch.nn.Module):
    """uint8 [N, 3, H, W] -> 16 features: 4x4 average pool, fixed random projection."""

    def __init__(self):
        super().__init__()
        self.register_buffer('w', torch.randn(3 * 16, 16, generator=torch.Generator().manual_seed(0)))

    def forward(self, x, return_features=True):
        x = torch.nn.functional.adaptive_avg_pool2d(x.float() / 255, 4).flatten(1)
        return x @ self.w.to(x.device)


def _zip(path, res=32, n=24):
    rs = np.random.RandomState(1)
    lab = []
    with zipfile.ZipFile(path, 'w') as z:
        for i in range(n):
            rel = f'p{i // 6:03d}/p{i // 6:03d}_{i % 6:05d}.pickle'
            img = np.clip(rs.randn(res, res) * 40 + 120 + 60 * np.sin(np.arange(res) / 3)[None], 0, 255)
            z.writestr(f'train/{rel}', pickle.dumps({'CT': img}))
            lab.append([rel, i % 2])
        z.writestr('train/dataset.json', json.dumps({'labels': lab}))


@pytest.mark.timeout(600)
def test_training_loop_end_to_end(tmp_path):
    import legacy
    import train_mi_multimodal as cli
    from metrics import metric_utils, frechet_inception_distance
    from metrics import metric_main_mi_multimodal as metric_main
    from torch_utils import misc
    zp = tmp_path / 'claro.zip'
    _zip(zp)
    metric_utils.register_detector(frechet_inception_distance.DETECTOR_URL, _ProjDetector())

    @metric_main.register_metric
    def fid2k_test(opts):          # fid50k_full's code path with 2k generated images (test time)
        opts.dataset_kwargs.update(max_size=None, xflip=False)
        return dict(fid2k_test=frechet_inception_distance.compute_fid(opts, max_real=None, num_gen=2000))

    c, desc, outdir, _ = cli.build_config(outdir=str(tmp_path / 'runs'), cfg='stylegan2', data=str(zp), dataset='claro',
                                          modalities='CT', cond=True, gpus=1, batch=8, gamma=0.4096, mirror=True,
                                          cbase=256, cmax=32, map_depth=2, metrics='fid2k_test', kimg=1, snap=1, tick=1,
                                          glr=0.0025, dlr=0.0025, aug='ada', target=0.6)
    c.total_kimg, c.kimg_per_tick = 0.128, 0.064          # 16 iterations, 2 ticks
    c.ada_interval = 4
    cli.launch_training(c=c, desc=desc, outdir=outdir, dry_run=False)
    run = c.run_dir
    lines = [json.loads(s) for s in open(os.path.join(run, 'stats.jsonl'))]
    assert len(lines) == 3          # tick 0 after the first iteration, then two full ticks
    last = lines[-1]
    for name in ('Progress/kimg', 'Timing/sec_per_kimg', 'Loss/G/loss', 'Loss/D/loss', 'Loss/signs/real',
                 'Loss/r1_penalty', 'Loss/pl_penalty', 'Progress/augment', 'Timing/Gmain'):
        assert name in last, name
    assert abs(last['Progress/kimg']['mean'] - 0.128) < 1e-6 and np.isfinite(last['Loss/G/loss']['mean'])
    snaps = sorted(f for f in os.listdir(run) if f.startswith('network-snapshot-'))
    assert snaps and os.path.exists(os.path.join(run, 'fakes_init.png')) and os.path.exists(os.path.join(run, 'reals.png'))
    fids = [json.loads(s) for s in open(os.path.join(run, 'metric-CT-fid2k_test.jsonl'))]
    assert len(fids) == 3 and all(np.isfinite(f['results']['fid2k_test']) for f in fids)
    opts = json.load(open(os.path.join(run, 'training_options.json')))
    assert opts['batch_gpu'] == 8 and opts['augment_kwargs']['class_name'] == 'training.augment_mi.AugmentPipe'

    # resume from the last snapshot: the networks come back bit-identical
    with open(os.path.join(run, snaps[-1]), 'rb') as f:
        snap = legacy.load_network_pkl(f)
    c2, desc2, outdir2, _ = cli.build_config(outdir=str(tmp_path / 'runs2'), cfg='stylegan2', data=str(zp),
                                             dataset='claro', modalities='CT', cond=True, gpus=1, batch=8,
                                             gamma=0.4096, cbase=256, cmax=32, map_depth=2, metrics='none', kimg=1,
                                             resume=os.path.join(run, snaps[-1]))
    assert c2.resume_pkl.endswith(snaps[-1]) and c2.ada_kimg == 100 and c2.ema_rampup is None
    from training import networks_stylegan2 as net
    G = net.Generator(**{k: v for k, v in c2.G_kwargs.items() if k != 'class_name'}, c_dim=2, img_resolution=32,
                      img_channels=1)
    misc.copy_params_and_buffers(snap['G_ema'], G, require_all=True)
    for (n, a), (_, b) in zip(G.named_parameters(), snap['G_ema'].named_parameters()):
        assert torch.equal(a, b), n
    assert float(snap['augment_pipe'].p) >= 0
