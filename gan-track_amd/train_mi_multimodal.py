"""Train StyleGAN2-ADA on Claro / Pelvis slices on MI355X -- the reference's trainer CLI.

Drop-in for SG3/train_mi_multimodal.py:148-358: the same click flags with the same defaults and the same
resolution into the EasyDict `c` passed to training_loop_mi_multimodal.training_loop (written to
training_options.json), including the reference's quirks: --ada_kimg is parsed but not applied (:319),
--rotate_max is in degrees and divided by 360 (:313), the StyleGAN2 defaults of :290-296.  The same
configuration can come from a YAML file (engine/train.py).

Process model: one process per GPU.  With --gpus > 1 ranks are spawned and join a torch.distributed
group with backend 'nccl' (RCCL over xGMI; rendezvous on 127.0.0.1).  Nothing is posted over the network
(the reference's IFTTT notifications, :371-388, are not reproduced).
"""
import json
import os
import re
import socket
import tempfile

import click
import torch

import dnnlib


def parse_comma_separated_list(s):
    if isinstance(s, list):
        return s
    if s is None or s.lower() == 'none' or s == '':
        return []
    return s.split(',')


def init_dataset_kwargs(data, dtype, split, modalities):
    """(reference init_dataset_mi_multimodal_kwargs, :114-125)"""
    modalities = modalities.replace(' ', '').split(',') if isinstance(modalities, str) else list(modalities)
    kw = dnnlib.EasyDict(class_name='training.dataset_mi_multimodal.CustomImageFolderDataset', path=data, dtype=dtype,
                         use_labels=True, max_size=None, xflip=False, split=split, modalities=modalities)
    obj = dnnlib.util.construct_class_by_name(**kw)
    kw.resolution = obj.resolution
    kw.use_labels = obj.has_labels
    kw.max_size = len(obj)
    return kw, obj.name


DEFAULTS = dict(dtype='float32', modalities='MR_nonrigid_CT,MR_MR_T2', dataset='Pelvis_2.1', split='train',
                metrics_cache=False, cond=False, mirror=False, aug='ada', ada_kimg=500,
                aug_opts='xflip,xint,scale,rotate,aniso,xfrac', xint_max=0.05, rotate_max=3, xfrac_std=0.05,
                scale_std=0.05, aniso_std=0.05, allow_aug_debug_print=False, resume=None, freezed=0, p=0.2,
                target=0.6, batch_gpu=None, cbase=32768, cmax=512, glr=None, dlr=0.002, map_depth=None,
                mbstd_group=4, desc=None, metrics='fid50k_full', kimg=25000, tick=4, snap=50, seed=0, fp32=False,
                nobench=False, workers=3, dry_run=False, graphs=False)


def build_config(**kwargs):
    """click-flag dict -> (c, desc, outdir): SG3/train_mi_multimodal.py:233-356 restated."""
    opts = dnnlib.EasyDict(DEFAULTS)
    opts.update({k.replace('-', '_'): v for k, v in kwargs.items() if v is not None or k in ('resume',)})
    for k in ('outdir', 'cfg', 'data', 'gpus', 'batch', 'gamma'):
        if opts.get(k) is None:
            raise click.ClickException(f'--{k} is required')
    if opts.cfg != 'stylegan2':
        raise click.ClickException('--cfg: only stylegan2 is served (the StyleGAN3 configurations are out of scope)')
    opts.aug_opts = parse_comma_separated_list(opts.aug_opts)
    opts.metrics = parse_comma_separated_list(opts.metrics)
    c = dnnlib.EasyDict()
    c.G_kwargs = dnnlib.EasyDict(class_name=None, z_dim=512, w_dim=512, mapping_kwargs=dnnlib.EasyDict())
    c.D_kwargs = dnnlib.EasyDict(class_name='training.networks_stylegan2.Discriminator', block_kwargs=dnnlib.EasyDict(),
                                 mapping_kwargs=dnnlib.EasyDict(), epilogue_kwargs=dnnlib.EasyDict())
    c.G_opt_kwargs = dnnlib.EasyDict(class_name='torch.optim.Adam', betas=[0, 0.99], eps=1e-8)
    c.D_opt_kwargs = dnnlib.EasyDict(class_name='torch.optim.Adam', betas=[0, 0.99], eps=1e-8)
    c.loss_kwargs = dnnlib.EasyDict(class_name='training.loss.StyleGAN2Loss')
    c.data_loader_kwargs = dnnlib.EasyDict(pin_memory=True, prefetch_factor=2)
    try:
        c.training_set_kwargs, dataset_name = init_dataset_kwargs(opts.data, opts.dtype, opts.split, opts.modalities)
    except IOError as err:
        raise click.ClickException(f'--data: {err}')
    c.metrics_cache = opts.metrics_cache
    c.loss_kwargs.allow_aug_debug_print = opts.allow_aug_debug_print
    if opts.cond and not c.training_set_kwargs.use_labels:
        raise click.ClickException('--cond=True requires labels specified in dataset.json')
    c.training_set_kwargs.use_labels = opts.cond
    c.training_set_kwargs.xflip = opts.mirror
    c.num_gpus = opts.gpus
    c.batch_size = opts.batch
    c.batch_gpu = opts.batch_gpu or opts.batch // opts.gpus
    c.G_kwargs.channel_base = c.D_kwargs.channel_base = opts.cbase
    c.G_kwargs.channel_max = c.D_kwargs.channel_max = opts.cmax
    c.G_kwargs.mapping_kwargs.num_layers = 8 if opts.map_depth is None else opts.map_depth
    c.D_kwargs.block_kwargs.freeze_layers = opts.freezed
    c.D_kwargs.epilogue_kwargs.mbstd_group_size = opts.mbstd_group
    c.loss_kwargs.r1_gamma = opts.gamma
    c.G_opt_kwargs.lr = 0.002 if opts.glr is None else opts.glr
    c.D_opt_kwargs.lr = opts.dlr
    c.metrics = opts.metrics
    c.total_kimg = opts.kimg
    c.kimg_per_tick = opts.tick
    c.image_snapshot_ticks = c.network_snapshot_ticks = opts.snap
    c.random_seed = c.training_set_kwargs.random_seed = opts.seed
    c.data_loader_kwargs.num_workers = opts.workers
    c.graphs = bool(opts.graphs)
    if c.batch_size % c.num_gpus != 0:
        raise click.ClickException('--batch must be a multiple of --gpus')
    if c.batch_size % (c.num_gpus * c.batch_gpu) != 0:
        raise click.ClickException('--batch must be a multiple of --gpus times --batch-gpu')
    if c.batch_gpu < c.D_kwargs.epilogue_kwargs.mbstd_group_size:
        raise click.ClickException('--batch-gpu cannot be smaller than --mbstd')
    from metrics import metric_main_mi_multimodal as metric_main
    if any(not metric_main.is_valid_metric(m) for m in c.metrics):
        raise click.ClickException('\n'.join(['--metrics can only contain the following values:'] +
                                             metric_main.list_valid_metrics()))
    c.ema_kimg = c.batch_size * 10 / 32
    c.G_kwargs.class_name = 'training.networks_stylegan2.Generator'
    c.loss_kwargs.style_mixing_prob = 0.9
    c.loss_kwargs.pl_weight = 2
    c.G_reg_interval = 4
    c.G_kwargs.fused_modconv_default = 'inference_only'
    c.loss_kwargs.pl_no_weight_grad = True
    if opts.aug != 'noaug':
        c.augment_kwargs = dnnlib.EasyDict(class_name='training.augment_mi.AugmentPipe', **{a: 1 for a in opts.aug_opts})
        c.augment_kwargs.xint_max = opts.xint_max
        c.augment_kwargs.rotate_max = opts.rotate_max / 360
        c.augment_kwargs.xfrac_std = opts.xfrac_std
        c.augment_kwargs.scale_std = opts.scale_std
        c.augment_kwargs.aniso_std = opts.aniso_std
        if opts.aug == 'ada':
            c.ada_target = opts.target      # (--ada_kimg is parsed but not applied, as in the reference)
        if opts.aug == 'fixed':
            c.augment_p = opts.p
    if opts.resume is not None:
        c.resume_pkl = opts.resume
        c.ada_kimg = 100
        c.ema_rampup = None
        c.loss_kwargs.blur_init_sigma = 0
    if opts.fp32:
        c.G_kwargs.num_fp16_res = c.D_kwargs.num_fp16_res = 0
        c.G_kwargs.conv_clamp = c.D_kwargs.conv_clamp = None
    if opts.nobench:
        c.cudnn_benchmark = False
    mods = ','.join(opts.modalities.replace(' ', '').split(',')) if isinstance(opts.modalities, str) else ','.join(opts.modalities)
    s_aug = ','.join(opts.aug_opts) if opts.aug != 'noaug' else 'noaug'
    outdir = os.path.join(opts.outdir, opts.dataset, 'training-runs', f'{dataset_name}', mods)
    desc = (f'{dataset_name}-{opts.cfg}-gpus_{c.num_gpus}-batch_{c.batch_size}-gamma_{c.loss_kwargs.r1_gamma:g}'
            f'-dtype_{opts.dtype}-split_{opts.split}-modalities_{mods}-aug_{opts.aug}-aug_opts_{s_aug}')
    if opts.desc is not None:
        desc += f'-{opts.desc}'
    return c, desc, outdir, bool(opts.dry_run)


def subprocess_fn(rank, c, master_port):
    log = dnnlib.util.Logger(file_name=os.path.join(c.run_dir, 'log.txt'), file_mode='a', should_flush=True)
    from torch_utils import training_stats
    from training import training_loop_mi_multimodal
    if c.num_gpus > 1:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(master_port)
        torch.cuda.set_device(rank)
        torch.distributed.init_process_group('nccl', rank=rank, world_size=c.num_gpus,
                                             device_id=torch.device('cuda', rank))
    training_stats.init_multiprocessing(rank=rank, sync_device=torch.device('cuda', rank) if c.num_gpus > 1 else None)
    try:
        training_loop_mi_multimodal.training_loop(rank=rank, **c)
    finally:
        if c.num_gpus > 1:
            torch.distributed.destroy_process_group()
        log.close()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_training(c, desc, outdir, dry_run):
    """(reference :53-109)"""
    log = dnnlib.util.Logger(should_flush=True)
    try:
        _launch(c, desc, outdir, dry_run)
    finally:
        log.close()


def _launch(c, desc, outdir, dry_run):
    prev = [x for x in os.listdir(outdir) if os.path.isdir(os.path.join(outdir, x))] if os.path.isdir(outdir) else []
    ids = [int(m.group()) for m in (re.match(r'^\d+', x) for x in prev) if m is not None]
    c.run_dir = os.path.join(outdir, f'{max(ids, default=-1) + 1:05d}-{desc}')
    assert not os.path.exists(c.run_dir)
    print('\nTraining options:\n' + json.dumps(c, indent=2) + '\n')
    print(f'Output directory:    {c.run_dir}\nNumber of GPUs:      {c.num_gpus}\nBatch size:          {c.batch_size} images')
    print(f'Training duration:   {c.total_kimg} kimg\nDataset path:        {c.training_set_kwargs.path}')
    print(f'Modalities:          {c.training_set_kwargs.modalities}\nDataset size:        {c.training_set_kwargs.max_size} images')
    if dry_run:
        print('Dry run; exiting.')
        return
    os.makedirs(c.run_dir)
    with open(os.path.join(c.run_dir, 'training_options.json'), 'wt') as f:
        json.dump(c, f, indent=2)
    port = _free_port()
    with tempfile.TemporaryDirectory():
        if c.num_gpus == 1:
            subprocess_fn(0, c, port)
        else:
            torch.multiprocessing.spawn(fn=subprocess_fn, args=(c, port), nprocs=c.num_gpus)


@click.command()
@click.option('--outdir', metavar='DIR', required=True)
@click.option('--cfg', type=click.Choice(['stylegan3-t', 'stylegan3-r', 'stylegan2']), required=True)
@click.option('--data', metavar='[ZIP|DIR]', type=str, required=True)
@click.option('--dtype', type=str, default='float32')
@click.option('--modalities', type=str, default='MR_nonrigid_CT,MR_MR_T2', required=True)
@click.option('--dataset', type=str, default='Pelvis_2.1', required=True)
@click.option('--split', type=str, default='train', required=True)
@click.option('--metrics_cache', type=bool, default=False, required=True)
@click.option('--gpus', type=click.IntRange(min=1), required=True)
@click.option('--batch', type=click.IntRange(min=1), required=True)
@click.option('--gamma', type=click.FloatRange(min=0), required=True)
@click.option('--cond', type=bool, default=False)
@click.option('--mirror', type=bool, default=False)
@click.option('--aug', type=click.Choice(['noaug', 'ada', 'fixed']), default='ada')
@click.option('--ada_kimg', type=click.IntRange(min=1), default=500)
@click.option('--aug_opts', type=parse_comma_separated_list, default='xflip,xint,scale,rotate,aniso,xfrac')
@click.option('--xint_max', type=click.FloatRange(min=0, max=1), default=0.05)
@click.option('--rotate_max', type=click.IntRange(min=0, max=360), default=3)
@click.option('--xfrac_std', type=click.FloatRange(min=0, max=1), default=0.05)
@click.option('--scale_std', type=click.FloatRange(min=0, max=1), default=0.05)
@click.option('--aniso_std', type=click.FloatRange(min=0, max=1), default=0.05)
@click.option('--allow_aug_debug_print', type=bool, default=False)
@click.option('--resume', type=str)
@click.option('--freezed', type=click.IntRange(min=0), default=0)
@click.option('--p', type=click.FloatRange(min=0, max=1), default=0.2)
@click.option('--target', type=click.FloatRange(min=0, max=1), default=0.6)
@click.option('--batch-gpu', type=click.IntRange(min=1))
@click.option('--cbase', type=click.IntRange(min=1), default=32768)
@click.option('--cmax', type=click.IntRange(min=1), default=512)
@click.option('--glr', type=click.FloatRange(min=0))
@click.option('--dlr', type=click.FloatRange(min=0), default=0.002)
@click.option('--map-depth', type=click.IntRange(min=1))
@click.option('--mbstd-group', type=click.IntRange(min=1), default=4)
@click.option('--desc', type=str)
@click.option('--metrics', type=parse_comma_separated_list, default='fid50k_full')
@click.option('--kimg', type=click.IntRange(min=1), default=25000)
@click.option('--tick', type=click.IntRange(min=1), default=4)
@click.option('--snap', type=click.IntRange(min=1), default=50)
@click.option('--seed', type=click.IntRange(min=0), default=0)
@click.option('--fp32', type=bool, default=False)
@click.option('--nobench', type=bool, default=False)
@click.option('--workers', type=click.IntRange(min=1), default=3)
@click.option('--graphs', type=bool, default=False, help='replay each phase from a HIP graph (this build)')
@click.option('-n', '--dry-run', is_flag=True)
def main(**kwargs):
    c, desc, outdir, dry_run = build_config(**kwargs)
    launch_training(c=c, desc=desc, outdir=outdir, dry_run=dry_run)


if __name__ == '__main__':
    main()   # pylint: disable=no-value-for-parameter
