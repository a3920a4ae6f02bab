"""The training loop: ticks, statistics, snapshots, metrics around the iteration of training/trainer.py.

Drop-in for SG3/training/training_loop_mi_multimodal.py:126-496 (same keyword arguments, the `c` that
train_mi_multimodal.py / engine/train.py build): data, networks, optional resume, ADA, the phase
schedule, status line per tick with the reference's training_stats names (Progress/*, Timing/*,
Resources/*), stats.jsonl, image grids, network-snapshot-<kimg>.pkl (torch_utils/persistence.py format)
and FID per modality.

MI355X-first differences:
  * the whole training split is decoded once into HBM (dataset_mi_multimodal.DeviceImageCache) and
    batches are gathered on the device in the reference sampler's order -- no DataLoader workers;
  * the iteration runs through Trainer (fused HIP kernels, flat-buffer optimiser, bucketed RCCL
    exchange overlapped with the backward, optional HIP-graph replay: `graphs=True`);
  * nothing is sent over the network (the reference posts IFTTT notifications at start / stop, :240,:494).
"""
import copy
import json
import os
import time

import numpy as np
import psutil
import torch

import dnnlib
import legacy
from torch_utils import misc
from torch_utils import training_stats
from training.dataset_mi_multimodal import DeviceImageCache
from training.trainer import Trainer


def to_grey_tiles(images, low, hi):
    """[N, C, H, W] -> [N*C, 1, H, W] in [0, 255]: every modality channel becomes its own grey tile
    (reference convert_to_grayscale, :35-50)."""
    images = np.asarray(images, dtype=np.float32)
    n, c, h, w = images.shape
    return ((images - low) * (255 / (hi - low))).reshape(n * c, 1, h, w)


def setup_snapshot_image_grid(training_set, modalities, random_seed=0):
    """Grid of real samples for the fakes*.png snapshots (reference :55-98): grouped by label when there
    are labels; the width is a multiple of the number of modalities (one tile per modality)."""
    rnd = np.random.RandomState(random_seed)
    gw = int(np.clip(7680 // training_set.image_shape[2], 7, 32))
    gh = int(np.clip(4320 // training_set.image_shape[1], 4, 32))
    gw -= gw % len(modalities)
    if not training_set.has_labels:
        order = list(range(len(training_set)))
        rnd.shuffle(order)
        idx = [order[i % len(order)] for i in range(gw * gh // len(modalities))]
    else:
        groups = {}
        for i in range(len(training_set)):
            groups.setdefault(tuple(training_set.get_details(i).raw_label.flat[::-1]), []).append(i)
        keys = sorted(groups)
        for k in keys:
            rnd.shuffle(groups[k])
        idx = []
        for y in range(gh):
            g = groups[keys[y % len(keys)]]
            idx += [g[x % len(g)] for x in range(gw)]
            groups[keys[y % len(keys)]] = [g[(i + gw) % len(g)] for i in range(len(g))]
    images, labels, _ = zip(*[training_set[i] for i in idx])
    return (gw, gh), to_grey_tiles(np.stack(images), 0.0, 255.0), np.stack(labels)


def save_image_grid(img, fname, grid_size):
    """[gw*gh, 1, H, W] tiles in [0, 255] -> one grey PNG (reference :103-121)."""
    img = np.rint(np.asarray(img, dtype=np.float32)).clip(0, 255).astype(np.uint8)
    gw, gh = grid_size
    _n, c, h, w = img.shape
    img = img.reshape(gh, gw, c, h, w).transpose(0, 3, 1, 4, 2).reshape(gh * h, gw * w, c)
    try:
        import PIL.Image
    except ImportError:
        np.save(os.path.splitext(fname)[0] + '.npy', img)
        return
    PIL.Image.fromarray(img[:, :, 0], 'L').save(fname)


def _fake_grid(G_ema, grid_z, grid_c):
    with torch.no_grad():
        images = torch.cat([G_ema(z=z, c=c, noise_mode='const').float().cpu() for z, c in zip(grid_z, grid_c)])
    return to_grey_tiles(images.numpy(), -1.0, 1.0)


def training_loop(run_dir='.', training_set_kwargs={}, data_loader_kwargs={}, G_kwargs={}, D_kwargs={}, G_opt_kwargs={},
                  D_opt_kwargs={}, augment_kwargs=None, loss_kwargs={}, metrics=[], metrics_cache=False, random_seed=0,
                  num_gpus=1, rank=0, batch_size=4, batch_gpu=4, ema_kimg=10, ema_rampup=0.05, G_reg_interval=None,
                  D_reg_interval=16, augment_p=0, ada_target=None, ada_interval=4, ada_kimg=500, total_kimg=25000,
                  kimg_per_tick=4, image_snapshot_ticks=50, network_snapshot_ticks=50, resume_pkl=None, resume_kimg=0,
                  cudnn_benchmark=True, abort_fn=None, progress_fn=None, graphs=False, device=None, **_unused):
    start_time = time.time()
    device = torch.device('cuda', rank) if device is None else torch.device(device)
    np.random.seed(random_seed * num_gpus + rank)
    torch.manual_seed(random_seed * num_gpus + rank)
    torch.backends.cudnn.benchmark = cudnn_benchmark
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False

    # Data: decoded once into HBM, served in the reference sampler's order.
    if rank == 0:
        print('Loading training set...')
    training_set = dnnlib.util.construct_class_by_name(**training_set_kwargs)
    data = DeviceImageCache(training_set, device, batch_size // num_gpus, rank=rank, num_replicas=num_gpus,
                            seed=random_seed)
    if rank == 0:
        print(f'\nNum images:  {len(training_set)}\nImage shape: {training_set.image_shape}\n'
              f'Label shape: {training_set.label_shape}\n')
    modalities = training_set.modalities

    # Networks.
    if rank == 0:
        print('Constructing networks...')
    common = dict(c_dim=training_set.label_dim, img_resolution=training_set.resolution,
                  img_channels=training_set.num_channels)
    G = dnnlib.util.construct_class_by_name(**G_kwargs, **common).train().requires_grad_(False).to(device)
    D = dnnlib.util.construct_class_by_name(**D_kwargs, **common).train().requires_grad_(False).to(device)
    G_ema = copy.deepcopy(G).eval()
    if resume_pkl is not None and rank == 0:
        print(f'Resuming from "{resume_pkl}"')
        with open(resume_pkl, 'rb') as f:
            resume_data = legacy.load_network_pkl(f)
        for name, module in [('G', G), ('D', D), ('G_ema', G_ema)]:
            misc.copy_params_and_buffers(resume_data[name], module, require_all=False)

    # Augmentation.
    augment_pipe = None
    if augment_kwargs is not None and (augment_p > 0 or ada_target is not None):
        augment_pipe = dnnlib.util.construct_class_by_name(run_dir=run_dir, batch_size=batch_size, **augment_kwargs)
        augment_pipe = augment_pipe.train().requires_grad_(False).to(device)
        augment_pipe.p.copy_(torch.as_tensor(augment_p))

    # Replicas start identical.
    if num_gpus > 1:
        for module in (G, D, G_ema, augment_pipe):
            if module is not None:
                for t in misc.params_and_buffers(module):
                    torch.distributed.broadcast(t, src=0)

    loss = dnnlib.util.construct_class_by_name(device=device, G=G, D=D, augment_pipe=augment_pipe, **loss_kwargs)
    trainer = Trainer(G, D, G_ema, loss, G_opt_kwargs, D_opt_kwargs, G_reg_interval=G_reg_interval,
                      D_reg_interval=D_reg_interval, batch_size=batch_size, batch_gpu=batch_gpu, num_gpus=num_gpus,
                      rank=rank, device=device, ema_kimg=ema_kimg, ema_rampup=ema_rampup, augment_pipe=augment_pipe,
                      ada_target=ada_target, ada_interval=ada_interval, ada_kimg=ada_kimg,
                      phase_timing=(rank == 0 and device.type == 'cuda'))

    # Sample grid.
    grid_size = grid_z = grid_c = None
    if rank == 0 and image_snapshot_ticks is not None:
        grid_size, images, labels = setup_snapshot_image_grid(training_set, modalities)
        save_image_grid(images, os.path.join(run_dir, 'reals.png'), grid_size=grid_size)
        grid_z = torch.randn([labels.shape[0], G.z_dim], device=device).split(batch_gpu)
        grid_c = torch.from_numpy(labels).to(device).split(batch_gpu)
        save_image_grid(_fake_grid(G_ema, grid_z, grid_c), os.path.join(run_dir, 'fakes_init.png'), grid_size)

    stats_collector = training_stats.Collector(regex='.*')
    stats_jsonl = open(os.path.join(run_dir, 'stats.jsonl'), 'wt') if rank == 0 else None
    if rank == 0:
        print(f'Training for {total_kimg} kimg...\n')
    cur_nimg = resume_kimg * 1000
    trainer.cur_nimg = cur_nimg
    cur_tick = 0
    tick_start_nimg = cur_nimg
    tick_start_time = time.time()
    maintenance_time = tick_start_time - start_time
    if progress_fn is not None:
        progress_fn(0, total_kimg)
    n_phases = len(trainer.phases)
    while True:
        with torch.autograd.profiler.record_function('data_fetch'):
            real, real_c = next(data)
            phase_real_img, phase_real_c = real.split(batch_gpu), real_c.split(batch_gpu)
            all_gen_z = torch.randn([n_phases * batch_size, G.z_dim], device=device)
            all_gen_z = [z.split(batch_gpu) for z in all_gen_z.split(batch_size)]
            all_gen_c = [training_set.get_label(np.random.randint(len(training_set))) for _ in range(n_phases * batch_size)]
            all_gen_c = torch.from_numpy(np.stack(all_gen_c)).to(device)
            all_gen_c = [c.split(batch_gpu) for c in all_gen_c.split(batch_size)]
        trainer.graphs = graphs and trainer.batch_idx > 0      # capture after one eager iteration
        trainer.step(phase_real_img, phase_real_c, all_gen_z, all_gen_c)
        cur_nimg = trainer.cur_nimg

        done = cur_nimg >= total_kimg * 1000
        if not done and cur_tick != 0 and cur_nimg < tick_start_nimg + kimg_per_tick * 1000:
            continue

        # Status line (its fields also reported to training_stats, as the reference does).
        tick_end_time = time.time()
        r0 = training_stats.report0
        fields = [f"tick {r0('Progress/tick', cur_tick):<5d}", f"kimg {r0('Progress/kimg', cur_nimg / 1e3):<8.1f}",
                  f"time {dnnlib.util.format_time(r0('Timing/total_sec', tick_end_time - start_time)):<12s}",
                  f"sec/tick {r0('Timing/sec_per_tick', tick_end_time - tick_start_time):<7.1f}",
                  f"sec/kimg {r0('Timing/sec_per_kimg', (tick_end_time - tick_start_time) / max(cur_nimg - tick_start_nimg, 1) * 1e3):<7.2f}",
                  f"maintenance {r0('Timing/maintenance_sec', maintenance_time):<6.1f}",
                  f"cpumem {r0('Resources/cpu_mem_gb', psutil.Process(os.getpid()).memory_info().rss / 2**30):<6.2f}"]
        if device.type == 'cuda':
            fields += [f"gpumem {r0('Resources/peak_gpu_mem_gb', torch.cuda.max_memory_allocated(device) / 2**30):<6.2f}",
                       f"reserved {r0('Resources/peak_gpu_mem_reserved_gb', torch.cuda.max_memory_reserved(device) / 2**30):<6.2f}"]
            torch.cuda.reset_peak_memory_stats(device)
        fields += [f"augment {r0('Progress/augment', float(augment_pipe.p.cpu()) if augment_pipe is not None else 0):.3f}"]
        r0('Timing/total_hours', (tick_end_time - start_time) / 3600)
        r0('Timing/total_days', (tick_end_time - start_time) / 86400)
        if rank == 0:
            print(' '.join(fields), flush=True)

        if not done and abort_fn is not None and abort_fn():
            done = True
            if rank == 0:
                print('\nAborting...')

        if rank == 0 and image_snapshot_ticks is not None and (done or cur_tick % image_snapshot_ticks == 0):
            save_image_grid(_fake_grid(G_ema, grid_z, grid_c), os.path.join(run_dir, f'fakes{cur_nimg // 1000:06d}.png'),
                            grid_size)

        snapshot_pkl = snapshot_data = None
        if network_snapshot_ticks is not None and (done or cur_tick % network_snapshot_ticks == 0):
            snapshot_pkl = os.path.join(run_dir, f'network-snapshot-{cur_nimg // 1000:06d}.pkl')
            snapshot_data = legacy.save_network_pkl(snapshot_pkl if rank == 0 else None, G, D, G_ema, augment_pipe,
                                                    training_set_kwargs, num_gpus=num_gpus)

        if snapshot_data is not None and len(metrics) > 0:
            from metrics import metric_main_mi_multimodal as metric_main
            if rank == 0:
                print('Evaluating metrics...')
            for metric in metrics:
                for mode_idx, mode in enumerate(modalities):
                    res = metric_main.calc_metric(metric=metric, G=snapshot_data['G_ema'], dataset_kwargs=training_set_kwargs,
                                                  num_gpus=num_gpus, rank=rank, device=device, cache=metrics_cache,
                                                  mode_dict={'mode_name': mode, 'mode_idx': mode_idx})
                    if rank == 0:
                        metric_main.report_metric(res, mode=mode, run_dir=run_dir, snapshot_pkl=snapshot_pkl)
        del snapshot_data

        for ph in trainer.phases:
            value = []
            if ph.start_event is not None and ph.end_event is not None:
                ph.end_event.synchronize()
                value = ph.start_event.elapsed_time(ph.end_event)
            training_stats.report0('Timing/' + ph.name, value)
        stats_collector.update()
        stats_dict = stats_collector.as_dict()
        if stats_jsonl is not None:
            stats_jsonl.write(json.dumps(dict(stats_dict, timestamp=time.time())) + '\n')
            stats_jsonl.flush()
        if progress_fn is not None:
            progress_fn(cur_nimg // 1000, total_kimg)

        cur_tick += 1
        tick_start_nimg = cur_nimg
        tick_start_time = time.time()
        maintenance_time = tick_start_time - tick_end_time
        if done:
            break
    if stats_jsonl is not None:
        stats_jsonl.close()
    if rank == 0:
        print('\nExiting...')

