"""The trainer shell around the iteration (CPU): data path, snapshots, FID statistics, config surface, ADA.

  * training/dataset_mi_multimodal.py vs the reference's semantics (SG3/training/dataset_mi_multimodal.py:
    30-285): zip of per-slice pickles, split filter, modality stacking, labels from <split>/dataset.json,
    max_size, x-flip doubling; the safe unpickler refuses code; DeviceImageCache serves the reference
    sampler's order;
  * torch_utils/persistence.py + legacy.py: snapshot round trip, refusal of foreign code and of StyleGAN3;
  * metrics/: FeatureStats against numpy, rank interleaving, FID formula, the real-image quirk;
  * train_mi_multimodal.build_config for the Claro job's flags (SG3/train_mi_multimodal.py:233-356), the
    YAML entry (engine/train.py) giving the same `c`;
  * the ADA heuristic (SG3/training/training_loop_mi_multimodal.py:373-376) through training_stats.
"""
import io
import json
import os
import pickle
import zipfile

import numpy as np
import pytest
import torch



# ------------------------------------------------------------------------------------------- dataset
def _make_zip(path, modalities=('CT',), res=16, patients=3, slices=4, labels=True, evil=False):
    from synth_zip import make_zip
    names = make_zip(path, modalities=modalities, res=res, patients=patients, slices=slices, labels=labels)
    if evil:
        class Evil:
            def __reduce__(self):
                return (os.system, ('echo pwned',))
        with zipfile.ZipFile(path, 'a') as z:
            z.writestr('train/zzz/zzz_00000.pickle', pickle.dumps({'CT': Evil()}))
    return names


def _ds(path, **kw):
    from training.dataset_mi_multimodal import CustomImageFolderDataset
    args = dict(path=str(path), dtype='float32', split='train', modalities=['CT'], use_labels=True)
    args.update(kw)
    return CustomImageFolderDataset(**args)


def test_dataset_semantics(tmp_path):
    zp = tmp_path / 'claro.zip'
    names = _make_zip(zp, modalities=('CT', 'PET'))
    ds = _ds(zp, modalities=['PET', 'CT'])
    assert len(ds) == 12 and ds.image_shape == [2, 16, 16] and ds.resolution == 16 and ds.num_channels == 2
    assert ds.label_shape == [2] and ds.has_labels and ds.has_onehot_labels
    img, lab, fname = ds[5]
    assert fname == 'train/' + sorted(names)[5] and img.dtype == np.float32
    with zipfile.ZipFile(zp) as z:
        raw = pickle.loads(z.read(fname))
    assert np.array_equal(img[0], raw['PET'].astype(np.float32)) and np.array_equal(img[1], raw['CT'].astype(np.float32))
    p = int(fname.split('/')[1][1:])
    assert lab.tolist() == [1.0 - p % 2, float(p % 2)]
    fl = _ds(zp, modalities=['PET', 'CT'], xflip=True)
    assert len(fl) == 24 and np.array_equal(fl[12 + 5][0], img[:, :, ::-1])
    sub = _ds(zp, modalities=['PET', 'CT'], max_size=5, random_seed=3)
    assert len(sub) == 5 and list(sub._raw_idx) == sorted(sub._raw_idx)
    nolab = _ds(zp, use_labels=False)
    assert nolab.label_dim == 0 and not nolab.has_labels


def test_dataset_refuses_code(tmp_path):
    zp = tmp_path / 'evil.zip'
    _make_zip(zp, evil=True)
    ds = _ds(zp)
    with pytest.raises(pickle.UnpicklingError, match='refused'):
        ds[len(ds) - 1]


def test_device_cache_follows_sampler(tmp_path):
    from training.dataset_mi_multimodal import DeviceImageCache
    from torch_utils import misc
    zp = tmp_path / 'claro.zip'
    _make_zip(zp)
    ds = _ds(zp, xflip=True)
    for rank in (0, 1):
        cache = DeviceImageCache(ds, 'cpu', batch_size=5, rank=rank, num_replicas=2, seed=7)
        ref = iter(torch.utils.data.DataLoader(ds, sampler=misc.InfiniteSampler(ds, rank=rank, num_replicas=2, seed=7),
                                               batch_size=5))
        for _ in range(4):
            img, c = next(cache)
            rimg, rc, _ = next(ref)
            assert torch.equal(img, rimg.float() / 127.5 - 1) and torch.equal(c, rc)


# ------------------------------------------------------------------------------------------- snapshots
def _nets():
    from training import networks_stylegan2 as net, augment_mi
    torch.manual_seed(0)
    G = net.Generator(z_dim=16, c_dim=2, w_dim=16, img_resolution=16, img_channels=1, channel_base=64, channel_max=8,
                      mapping_kwargs=dict(num_layers=2))
    D = net.Discriminator(c_dim=2, img_resolution=16, img_channels=1, channel_base=64, channel_max=8)
    A = augment_mi.AugmentPipe(run_dir=None, batch_size=4, xflip=1, rotate=1, scale=1)
    with torch.no_grad():
        for p in list(G.parameters()) + list(D.parameters()):
            p.add_(torch.randn_like(p))
        A.p.fill_(0.25)
    return G, D, A


def test_snapshot_round_trip(tmp_path):
    import legacy
    G, D, A = _nets()
    path = tmp_path / 'network-snapshot-000004.pkl'
    legacy.save_network_pkl(str(path), G, D, G, A, dict(path='claro.zip', modalities=['CT']))
    with open(path, 'rb') as f:
        d = legacy.load_network_pkl(f)
    for key, mod in [('G', G), ('D', D), ('G_ema', G)]:
        got = dict(list(d[key].named_parameters()) + list(d[key].named_buffers()))
        for n, t in list(mod.named_parameters()) + list(mod.named_buffers()):
            assert torch.equal(got[n], t.detach()), (key, n)
        assert not d[key].training
    assert float(d['augment_pipe'].p) == 0.25 and d['training_set_kwargs']['modalities'] == ['CT']
    assert d['G'].init_kwargs.channel_base == 64 and d['G'].init_kwargs.mapping_kwargs == dict(num_layers=2)
    with open(path, 'rb') as f:
        d16 = legacy.load_network_pkl(f, force_fp16=True)
    assert d16['G'].init_kwargs.num_fp16_res == 4 and d16['G'].init_kwargs.conv_clamp == 256


def test_snapshot_refuses_code_and_sg3(tmp_path):
    import legacy
    from torch_utils import persistence

    class Evil:
        def __reduce__(self):
            return (os.system, ('echo pwned',))
    with pytest.raises(pickle.UnpicklingError, match='refused'):
        legacy.load_network_pkl(io.BytesIO(pickle.dumps(dict(G=Evil()))))
    # a persistent object whose source is a StyleGAN3 network: not executed, refused
    meta = dict(type='class', version=6, module_src='class SynthesisInput: pass\nimport os; os.system("echo")',
                class_name='Generator', state={})
    with pytest.raises(pickle.UnpicklingError, match='StyleGAN3'):
        persistence._reconstruct_persistent_obj(meta)
    # a persistent object of a class this build does not have
    meta = dict(type='class', version=6, module_src='', class_name='NotANetwork', state={})
    with pytest.raises(pickle.UnpicklingError):
        persistence._reconstruct_persistent_obj(meta)


# ------------------------------------------------------------------------------------------- metrics
def test_feature_stats_and_fid():
    import scipy.linalg
    from metrics import metric_utils, frechet_inception_distance as fid
    rs = np.random.RandomState(1)
    feats = rs.randn(103, 12).astype(np.float32) * rs.rand(12).astype(np.float32)
    s = metric_utils.FeatureStats(capture_mean_cov=True, max_items=97)
    for b in range(0, 103, 10):
        s.append_torch(torch.from_numpy(feats[b:b + 10]))
    mean, cov = s.get_mean_cov()
    x = feats[:97].astype(np.float64)
    assert s.num_items == 97
    assert np.allclose(mean, x.mean(0), atol=1e-12) and np.allclose(cov, np.cov(x.T, bias=True), atol=1e-10)
    # two ranks, interleaved stream (rank r holds items k*2 + r), truncated at 15 items
    parts = []
    for rank in (0, 1):
        sr = metric_utils.FeatureStats(capture_mean_cov=True, max_items=15)
        for b in range(0, 16, 4):     # the global stream in batches of 4 per rank
            glob = feats[2 * b:2 * b + 8]
            sr.append_torch(torch.from_numpy(glob[rank::2]), num_gpus=2, rank=rank)
        assert sr.num_items == 15
        parts.append(sr)
    tot = parts[0].raw_mean + parts[1].raw_mean
    assert np.allclose(tot.numpy(), feats[:15].astype(np.float64).sum(0), atol=1e-9)
    # FID formula
    a, b = rs.randn(500, 6), rs.randn(400, 6) * 1.3 + 0.2
    m1, s1, m2, s2 = a.mean(0), np.cov(a.T), b.mean(0), np.cov(b.T)
    want = np.sum((m1 - m2) ** 2) + np.trace(s1 + s2 - 2 * np.real(scipy.linalg.sqrtm(s1 @ s2)))
    assert abs(fid.fid_from_stats(m1, s1, m2, s2) - want) < 1e-9 and abs(fid.fid_from_stats(m1, s1, m1, s1)) < 1e-6


def test_real_image_quirk():
    from metrics import metric_utils
    x = torch.tensor([[[[0.0, 100.5], [254.0, 3.2]]]])
    y = metric_utils.real_images_to_uint8_quirk(x)            # max != 255: *255, clamp, uint8
    assert y.dtype == torch.uint8 and y.flatten().tolist() == [0, 255, 255, 255]
    x2 = torch.tensor([[[[0.0, 100.5], [255.0, 3.2]]]])
    assert torch.equal(metric_utils.real_images_to_uint8_quirk(x2), x2)   # max == 255: unchanged float


# ------------------------------------------------------------------------------------------- config surface
CLARO_FLAGS = dict(outdir=None, cfg='stylegan2', data=None, dataset='claro', dtype='float32', modalities='CT',
                   split='train', metrics_cache=True, cond=True, gpus=2, batch=32, map_depth=8, glr=0.0025,
                   dlr=0.0025, cbase=16384, gamma=0.4096, mirror=True, aug='ada', ada_kimg=77,
                   aug_opts='xflip,xint,scale,rotate,aniso,xfrac', xint_max=0.05, rotate_max=3, xfrac_std=0.05,
                   scale_std=0.05, aniso_std=0.05, target=0.6, metrics='fid50k_full')


def test_build_config_claro(tmp_path):
    import train_mi_multimodal as cli
    zp = tmp_path / 'claro.zip'
    _make_zip(zp)
    c, desc, outdir, dry = cli.build_config(**dict(CLARO_FLAGS, outdir=str(tmp_path / 'runs'), data=str(zp)))
    assert c.batch_gpu == 16 and c.num_gpus == 2 and c.ema_kimg == 10
    assert c.G_kwargs.class_name == 'training.networks_stylegan2.Generator' and c.G_kwargs.mapping_kwargs.num_layers == 8
    assert c.G_kwargs.channel_base == c.D_kwargs.channel_base == 16384
    assert c.G_opt_kwargs.lr == 0.0025 and c.D_opt_kwargs.lr == 0.0025 and c.G_reg_interval == 4
    assert c.loss_kwargs.r1_gamma == 0.4096 and c.loss_kwargs.pl_weight == 2 and c.loss_kwargs.style_mixing_prob == 0.9
    assert c.loss_kwargs.pl_no_weight_grad and c.G_kwargs.fused_modconv_default == 'inference_only'
    assert c.augment_kwargs.rotate_max == 3 / 360 and c.augment_kwargs.xflip == 1 and c.ada_target == 0.6
    assert 'ada_kimg' not in c                                    # parsed, not applied (reference :319)
    assert c.training_set_kwargs.use_labels and c.training_set_kwargs.xflip and c.training_set_kwargs.max_size == 12
    assert c.training_set_kwargs.modalities == ['CT'] and c.metrics == ['fid50k_full']
    assert desc.startswith('claro-stylegan2-gpus_2-batch_32-gamma_0.4096') and outdir.endswith(os.path.join('claro', 'training-runs', 'claro', 'CT'))
    cli.launch_training(c=c, desc=desc, outdir=outdir, dry_run=True)     # prints, writes nothing
    assert not os.path.exists(outdir)


def test_yaml_entry_matches_flags(tmp_path):
    import yaml
    import train_mi_multimodal as cli
    from engine import train as engine_train
    zp = tmp_path / 'claro.zip'
    _make_zip(zp)
    flags = dict(CLARO_FLAGS, outdir=str(tmp_path / 'runs'), data=str(zp))
    block = {k.replace('_', '-') if k == 'map_depth' else k: v for k, v in flags.items()}
    block['aug_opts'] = flags['aug_opts'].split(',')
    cfgf = tmp_path / 'claro.yaml'
    cfgf.write_text(yaml.safe_dump({'seed': 5, 'trainer_gan': block}))
    opts = engine_train.options_from_yaml(str(cfgf), ['kimg=123'])
    c1, d1, o1, _ = cli.build_config(**opts)
    c2, d2, o2, _ = cli.build_config(**dict(flags, seed=5, kimg=123))
    assert json.dumps(c1, sort_keys=True) == json.dumps(c2, sort_keys=True) and (d1, o1) == (d2, o2)
    with pytest.raises(SystemExit, match='not trainer flags'):
        cfgf.write_text(yaml.safe_dump({'trainer_gan': dict(block, w_dimm=3)}))
        engine_train.options_from_yaml(str(cfgf))


# ------------------------------------------------------------------------------------------- ADA heuristic
def test_ada_heuristic_moves_p():
    """p += sign(E[sign(D(real))] - target) * B * I / (ada_kimg * 1000), clamped at 0, every I iterations
    (reference :373-376); the signs flow through training_stats.report -> Collector, as in the reference."""
    from oracle import sg2_oracle as O
    from training import loss as loss_mod
    from training.trainer import Trainer
    from torch_utils import training_stats
    torch.manual_seed(0)
    G = O.Generator(z_dim=16, c_dim=0, w_dim=16, img_resolution=16, img_channels=1, channel_base=64, channel_max=8,
                    mapping_kwargs=dict(num_layers=2)).train().requires_grad_(False)
    D = O.Discriminator(c_dim=0, img_resolution=16, img_channels=1, channel_base=64, channel_max=8,
                        epilogue_kwargs=dict(mbstd_group_size=2)).train().requires_grad_(False)
    aug = O.AugmentPipe(xflip=1, rotate=1)
    aug.p.fill_(0.01)
    loss = loss_mod.StyleGAN2Loss(device=torch.device('cpu'), G=G, D=D, augment_pipe=aug, r1_gamma=1,
                                  style_mixing_prob=0, pl_weight=0)
    opt = dict(class_name='torch.optim.Adam', lr=0.002, betas=[0, 0.99], eps=1e-8)
    B, I, K = 4, 2, 3
    tr = Trainer(G, D, copy_module(G), loss, opt, opt, batch_size=B, batch_gpu=B, device=torch.device('cpu'),
                 augment_pipe=aug, ada_target=0.6, ada_interval=I, ada_kimg=K)
    watch = training_stats.Collector(regex='Loss/signs/real')
    p_hist = []
    for it in range(2 * I):
        real = torch.rand([B, 1, 16, 16]) * 2 - 1
        z = torch.randn([4, B, 16])
        c = torch.zeros([4, B, 0])
        p_before = float(aug.p)
        tr.step([real], [torch.zeros([B, 0])], [[z[i]] for i in range(4)], [[c[i]] for i in range(4)])
        p_hist.append((p_before, float(aug.p)))
        if (it + 1) % I == 0:
            watch.update()
            mean_sign = watch['Loss/signs/real']
            want = max(p_before + np.sign(mean_sign - 0.6) * (B * I) / (K * 1000), 0)
            assert abs(float(aug.p) - want) < 1e-7, (it, float(aug.p), want)
        else:
            assert p_hist[-1][0] == p_hist[-1][1]
    assert any(a != b for a, b in p_hist)


def copy_module(m):
    import copy
    return copy.deepcopy(m).eval()





def test_stats_board_refuses_growth_after_capture():
    """training_stats keeps one device table per device; captured phase graphs hold pointers into it.  A new
    statistic name that needs a bigger table after a capture must raise instead of silently re-allocating
    (the captured reports -- Loss/signs/real, which drives ADA's p -- would go to the old table)."""
    from torch_utils import training_stats as ts
    b = ts._Board()
    b.table(torch.device('cpu'))
    for i in range(b.capacity):
        b.row(f'stat{i}')
    b.row('stat0')                       # existing names never grow the table
    b.captured = True
    with pytest.raises(RuntimeError, match='after a HIP graph was captured'):
        b.row('one_too_many')
    assert 'one_too_many' not in b.rows and len(b.rows) == b.capacity
    b.captured = False
    b.row('one_too_many')                # before any capture the board grows, keeping its rows
    assert b.tables[torch.device('cpu')].shape[0] == b.capacity == 512


# ------------------------------------------------------------------------- parity with the reference's own runs
# tests/golden/shell_ref.npz was written by the REFERENCE (tests/golden/make_shell_golden.py) on the same
# synthetic zips (tests/golden/synth_zip.py): bit-exact for the index / byte work, float64 rounding for FID.
def _shell_ref():
    import ast
    z = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'shell_ref.npz'), allow_pickle=False)
    return z, ast.literal_eval(str(z['zips'])), ast.literal_eval(str(z['datasets']))


def _ref_zips(tmp_path, zips):
    from synth_zip import make_zip
    paths = {}
    for name, kw in zips.items():
        paths[name] = str(tmp_path / f'{name}.zip')
        make_zip(paths[name], **kw)
    return paths


def _dataset_kwargs(zpath, kw):
    import dnnlib
    d = dict(class_name='training.dataset_mi_multimodal.CustomImageFolderDataset', path=zpath, dtype='float32',
             split='train', use_labels=False, xflip=False, max_size=None)
    d.update(kw)
    return dnnlib.EasyDict(d)


def test_data_path_matches_reference(tmp_path):
    """Every item (file name, label, CRC of the decoded float32 image after the x-flip), max_size / xflip
    indexing, the split's substring file selection, InfiniteSampler's index streams and the first batches the
    training loop consumes (DeviceImageCache vs the reference's DataLoader + / 127.5 - 1), bit for bit against
    the reference's own run (SG3/training/dataset_mi_multimodal.py:30-285, torch_utils/misc.py:111-142)."""
    import zlib
    import dnnlib
    from torch_utils import misc
    from training.dataset_mi_multimodal import DeviceImageCache
    z, zips, datasets = _shell_ref()
    paths = _ref_zips(tmp_path, zips)
    crc = lambda a: zlib.crc32(np.ascontiguousarray(a).tobytes())   # noqa: E731
    for name, (zname, kw) in datasets.items():
        ds = dnnlib.util.construct_class_by_name(**_dataset_kwargs(paths[zname], kw))
        assert len(ds) == int(z[f'ds/{name}/len']), name
        assert np.array_equal(ds._raw_idx, z[f'ds/{name}/raw_idx']) and np.array_equal(ds._xflip, z[f'ds/{name}/xflip'])
        items = [ds[i] for i in range(len(ds))]
        assert [it[2] for it in items] == z[f'ds/{name}/fnames'].tolist(), name
        assert np.array_equal(np.stack([it[1] for it in items]).astype(np.float32), z[f'ds/{name}/labels']), name
        assert [crc(it[0]) for it in items] == z[f'ds/{name}/crc'].tolist(), name
        for key in [k for k in z.files if k.startswith(f'ds/{name}/sampler/')]:
            rank, nrep, seed = map(int, key.rsplit('/', 1)[1].split('_'))
            it = iter(misc.InfiniteSampler(ds, rank=rank, num_replicas=nrep, seed=seed))
            assert [next(it) for _ in range(100)] == z[key].tolist(), key
        for key in [k for k in z.files if k.startswith(f'ds/{name}/batches/')]:
            rank, nrep, seed = map(int, key.rsplit('/', 1)[1].split('_'))
            cache = DeviceImageCache(ds, 'cpu', batch_size=5, rank=rank, num_replicas=nrep, seed=seed)
            got = [[crc(img.numpy()), crc(c.numpy())] for img, c in (next(cache) for _ in range(3))]
            assert got == z[key].tolist(), key
    assert int(z['ds/quirk/len']) == 14      # 12 train slices + the 2 'val/retrain*' ones the substring rule admits


@pytest.mark.parametrize('case', ['ct_peak', 'pelvis'])
def test_fid_pipeline_matches_reference(tmp_path, case):
    """compute_fid and both feature-statistics passes (real: the x 255 / uint8 quirk or the pass-through, per
    modality; generated: latents, labels from the dataset, uint8 conversion) against the reference's own run with
    the same stub detector and generator (tests/golden/stub_metric.py) and seeds: moments to float64 rounding,
    FID to 1e-9 relative (SG3/metrics/metric_utils.py:201-306, frechet_inception_distance.py:19-40).  The real
    Inception network is not available offline, so FID-50k itself stays unmeasured here."""
    import ast
    from metrics import metric_utils, frechet_inception_distance as fidm
    from stub_metric import StubDetector, StubGenerator
    z, zips, _ = _shell_ref()
    paths = _ref_zips(tmp_path, zips)
    args = ast.literal_eval(str(z[f'fid/{case}/args']))
    if case == 'ct_peak':
        dkw = _dataset_kwargs(paths['ct_peak'], dict(modalities=['CT'], use_labels=True))
        G = StubGenerator(c_dim=2, img_channels=1)
    else:
        dkw = _dataset_kwargs(paths['pelvis'], dict(modalities=['MR_MR_T2', 'MR_nonrigid_CT']))
        G = StubGenerator(c_dim=0, img_channels=2)
    metric_utils.register_detector(fidm.DETECTOR_URL, StubDetector(res=16))
    mode = args['mode']

    def opts():
        return metric_utils.MetricOptions(G=G, dataset_kwargs=dkw, num_gpus=1, rank=0, device=torch.device('cpu'),
                                          cache=False, mode_dict=mode)
    np.random.seed(5)
    torch.manual_seed(6)
    fid = fidm.compute_fid(opts(), args['max_real'], args['num_gen'])
    np.random.seed(5)
    torch.manual_seed(6)
    kw = dict(detector_url=fidm.DETECTOR_URL, detector_kwargs=dict(return_features=True), mode_dict=mode,
              capture_mean_cov=True)
    mr, sr = metric_utils.compute_feature_stats_for_dataset(opts=opts(), rel_lo=0, rel_hi=0, max_items=args['max_real'],
                                                            **kw).get_mean_cov()
    mg, sg = metric_utils.compute_feature_stats_for_generator(opts=opts(), rel_lo=0, rel_hi=1, max_items=args['num_gen'],
                                                              **kw).get_mean_cov()
    for k, v in dict(mu_real=mr, sigma_real=sr, mu_gen=mg, sigma_gen=sg).items():
        ref = z[f'fid/{case}/{k}']
        assert np.allclose(v, ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max()), k
    ref_fid = float(z[f'fid/{case}/fid'])
    assert abs(fid - ref_fid) <= 1e-9 * abs(ref_fid), (fid, ref_fid)


REF_SG3 = '/root/reference/src/models/stylegan3'


@pytest.mark.skipif(not os.path.isdir(REF_SG3), reason='needs the reference tree (build container only)')
def test_snapshot_from_reference(tmp_path):
    """A network-snapshot pickle written by the REFERENCE's own persistence / pickling (tests/golden/ref_snapshot.py,
    run in a subprocess on the reference tree) loads with this build's legacy.load_network_pkl -- without executing
    the source it embeds -- into this build's classes, every parameter and buffer bit-equal, the constructor
    arguments and the augment pipe's p preserved (SG3/torch_utils/persistence.py:35-130, legacy.py:22-58).  The
    pickle embeds the reference's source, so it is produced here and never committed."""
    import subprocess
    import sys
    import legacy
    from training import networks_stylegan2 as net, augment_mi
    pkl, npz = tmp_path / 'network-snapshot-000000.pkl', tmp_path / 'ref_state.npz'
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE='1',
               PYTHONPATH=os.pathsep.join([REF_SG3, os.path.join(os.path.dirname(__file__), 'golden')]))
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), 'golden', 'ref_snapshot.py'), str(pkl),
                        str(npz)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    ref = np.load(npz, allow_pickle=False)
    with open(pkl, 'rb') as f:
        data = legacy.load_network_pkl(f)
    assert isinstance(data['G'], net.Generator) and isinstance(data['D'], net.Discriminator)
    assert isinstance(data['G_ema'], net.Generator) and isinstance(data['augment_pipe'], augment_mi.AugmentPipe)
    assert data['training_set_kwargs']['modalities'] == ['CT']
    import ast
    n_checked = 0
    for key in ('G', 'D', 'G_ema', 'augment_pipe'):
        got = dict(list(data[key].named_parameters()) + list(data[key].named_buffers()))
        want = {k.split('/', 1)[1]: ref[k] for k in ref.files if k.startswith(key + '/') and not k.endswith('init_kwargs')}
        assert set(got) == set(want), (key, set(got) ^ set(want))
        for n, v in want.items():
            assert got[n].dtype == torch.from_numpy(v).dtype and np.array_equal(got[n].detach().numpy(), v), (key, n)
            n_checked += 1
        assert not data[key].training
        assert dict(data[key].init_kwargs) == ast.literal_eval(str(ref[f'{key}/init_kwargs'])), key
    assert float(data['augment_pipe'].p) == 0.375 and n_checked > 100


def test_metric_registry(tmp_path, capsys):
    """metric_main_mi_multimodal (SG3/metrics/metric_main_mi_multimodal.py:27-95): registration, calc_metric's result
    record, report_metric's JSON line in <run_dir>/metric-<modality>-<metric>.jsonl with the snapshot path relative
    to the run directory, and unknown names refused."""
    import json
    import os
    import torch
    from metrics import metric_main_mi_multimodal as metric_main

    assert {'fid50k_full', 'fid50k'} <= set(metric_main.list_valid_metrics())

    @metric_main.register_metric
    def unit_metric(opts):
        assert opts.num_gpus == 1 and opts.dataset_kwargs.path == 'x.zip'
        return {'unit_metric': 1.5}

    assert metric_main.is_valid_metric('unit_metric') and not metric_main.is_valid_metric('nope')
    res = metric_main.calc_metric(metric='unit_metric', dataset_kwargs={'path': 'x.zip'}, device=torch.device('cpu'))
    assert res.results.unit_metric == 1.5 and res.metric == 'unit_metric' and res.num_gpus == 1
    assert isinstance(res.total_time_str, str)
    metric_main.report_metric(res, mode='CT', run_dir=str(tmp_path), snapshot_pkl=str(tmp_path / 'network-snapshot-000001.pkl'))
    line = json.loads(open(os.path.join(tmp_path, 'metric-CT-unit_metric.jsonl')).read().strip())
    assert line['results'] == {'unit_metric': 1.5} and line['mode'] == 'CT'
    assert line['snapshot_pkl'] == 'network-snapshot-000001.pkl' and 'timestamp' in line
    assert json.loads(capsys.readouterr().out.strip().splitlines()[-1]) == line
    with pytest.raises(AssertionError):
        metric_main.calc_metric(metric='nope')
