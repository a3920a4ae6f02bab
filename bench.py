"""Benchmark: StyleGAN2-ADA training throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1] per GPU; configs[2] at N=8): the Claro job of the reference
(src/bash/claro-*.sh:18 -> SG3/train_mi_multimodal.py): 256x256 1-channel images, conditional
(c_dim=2), cbase 16384, cmax 512, mapping depth 8, z=w=512, mbstd group 4, batch 32 per GPU,
gamma 0.4096, PL weight 2 (every 4 iterations, half batch), R1 every 16, style mixing 0.9,
lazy-reg Adam (lr 0.0025, betas (0, 0.99)), EMA, ADA pipe with the job's geometric ops at fixed
p = 0.2, fp16 at the 4 highest resolutions (num_fp16_res=4, conv_clamp 256), the rest fp32.
Synthetic data (no dataset in the container): reals ~ U(-1,1) resident in HBM, z ~ N(0,1) drawn
on the device each iteration, random one-hot labels; networks randomly initialised (seed 0).

A "step" = one training iteration with the reference's phase schedule (Gmain + Dmain every step,
Greg every 4th, Dreg every 16th, gradient all-reduce, Adam, EMA, ADA); the phase counter is reset
at the start of the timed region, so K steps contain the schedule's phases as they fall from step 0:
K = 16 is exactly one cycle (4 Greg, 1 Dreg); K = 20 has 5 Greg and 2 Dreg (10 % Dreg steps against the
schedule's 6.25 %, so a 20-step value is slightly pessimistic).
value = images processed by all ranks / max-over-ranks wall time of the K timed steps.

Extra fields: `roofline` for the dominant kernel (the MFMA implicit-GEMM convolution of the 256^2
layers -- the top-resolution synthesis layer at the run's own batch, so C4 / C5 report their 512^2 C=64 /
1024^2 C=32 layers -- timed with HIP events on the launching stream after the timed region) and `cpu_baseline`
(the CPU oracle restatement of the same iteration on the host cores, bounded sample, rank 0, N=1).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, 'gan-track_amd'), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

MFMA_PEAK_FP16 = 2500.0   # TFLOP/s dense (MI355X_MICROARCH.md, Peak BF16/FP16 MFMA)
HBM_PEAK = 8000.0         # GB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=16)
    ap.add_argument('--warmup', type=int, default=4)
    ap.add_argument('--res', type=int, default=256)
    ap.add_argument('--batch-gpu', type=int, default=32)
    ap.add_argument('--cbase', type=int, default=16384)
    ap.add_argument('--img-channels', type=int, default=1)
    ap.add_argument('--c-dim', type=int, default=2)
    ap.add_argument('--map-depth', type=int, default=8)
    ap.add_argument('--fp16-dtype', default='fp16', choices=['fp16', 'bf16'])
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-roofline', action='store_true')
    ap.add_argument('--phase-timing', action='store_true')
    ap.add_argument('--graphs', default='auto', choices=['auto', 'on', 'off'],
                    help='HIP-graph replay of each phase, the bucket all_reduces captured into the phase graphs with '
                         'several GPUs (auto: on, after a capture probe of an RCCL all_reduce agrees on every rank; '
                         'otherwise the eager path, whose bucketed all_reduces overlap the backward from hooks)')
    ap.add_argument('--no-graphs', action='store_true', help='same as --graphs off')
    return ap.parse_args()


def rccl_graph_ok(device, world):
    """Can this stack capture the trainer's exchange pattern (an async RCCL all_reduce joined with wait())
    into a HIP graph and replay it correctly?  Every rank captures; the replay runs only if all ranks captured
    (an eager MIN over the ranks' flags, so no rank replays a collective the others will not join); the
    replayed value is checked and agreed on the same way.  False -> the bench stays on the eager path."""
    dist = torch.distributed

    def agree(flag):
        t = torch.tensor([1.0 if flag else 0.0], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return float(t) == 1.0

    src = torch.ones(4096, device=device)
    dist.all_reduce(src.clone())                      # communicator warm-up, eager
    torch.cuda.synchronize(device)
    g, ok = torch.cuda.CUDAGraph(), True
    try:
        with torch.cuda.graph(g):
            y = src * 2
            work = dist.all_reduce(y, async_op=True)
            work.wait()
            z = y + 1
    except Exception as e:                            # noqa: BLE001 (any capture failure -> eager path)
        print(f'[bench] RCCL graph capture failed: {e!r}', flush=True)
        ok = False
    if not agree(ok):
        return False
    src.fill_(3.0)
    g.replay()
    torch.cuda.synchronize(device)
    ok = bool((z == 6.0 * world + 1).all())
    return agree(ok)


def build(args, device, rank, num_gpus):
    import dnnlib
    from training import networks_stylegan2 as net, augment_mi, loss as loss_mod, trainer as trainer_mod
    fp16_dtype = torch.float16 if args.fp16_dtype == 'fp16' else torch.bfloat16
    torch.manual_seed(0)
    G = net.Generator(z_dim=512, c_dim=args.c_dim, w_dim=512, img_resolution=args.res, img_channels=args.img_channels,
                      channel_base=args.cbase, channel_max=512, num_fp16_res=4, conv_clamp=256,
                      fused_modconv_default='inference_only', fp16_dtype=fp16_dtype,
                      mapping_kwargs=dict(num_layers=args.map_depth))
    D = net.Discriminator(c_dim=args.c_dim, img_resolution=args.res, img_channels=args.img_channels,
                          channel_base=args.cbase, channel_max=512, num_fp16_res=4, conv_clamp=256,
                          block_kwargs=dict(fp16_dtype=fp16_dtype), epilogue_kwargs=dict(mbstd_group_size=4))
    G = G.train().requires_grad_(False).to(device)
    D = D.train().requires_grad_(False).to(device)
    G_ema = net.Generator(z_dim=512, c_dim=args.c_dim, w_dim=512, img_resolution=args.res,
                          img_channels=args.img_channels, channel_base=args.cbase, channel_max=512, num_fp16_res=4,
                          conv_clamp=256, fp16_dtype=fp16_dtype,
                          mapping_kwargs=dict(num_layers=args.map_depth)).eval().requires_grad_(False).to(device)
    G_ema.load_state_dict(G.state_dict())
    aug = augment_mi.AugmentPipe(run_dir=None, batch_size=args.batch_gpu * num_gpus, xflip=1, xint=1, scale=1,
                                 rotate=1, aniso=1, xfrac=1, xint_max=0.05, rotate_max=3 / 360, xfrac_std=0.05,
                                 scale_std=0.05, aniso_std=0.05).train().requires_grad_(False).to(device)
    aug.p.copy_(torch.as_tensor(0.2))
    if num_gpus > 1:
        for m in (G, D, G_ema, aug):
            for t in list(m.parameters()) + list(m.buffers()):
                torch.distributed.broadcast(t, src=0)
    loss = loss_mod.StyleGAN2Loss(device=device, G=G, D=D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9,
                                  pl_weight=2, pl_no_weight_grad=True)
    opt = dnnlib.EasyDict(class_name='torch.optim.Adam', lr=0.0025, betas=[0, 0.99], eps=1e-8)
    B = args.batch_gpu * num_gpus
    tr = trainer_mod.Trainer(G, D, G_ema, loss, opt, dnnlib.EasyDict(opt), G_reg_interval=4, D_reg_interval=16,
                             batch_size=B, batch_gpu=args.batch_gpu, num_gpus=num_gpus, rank=rank, device=device,
                             ema_kimg=B * 10 / 32, augment_pipe=aug, ada_target=None,
                             phase_timing=args.phase_timing)
    return tr


def make_inputs(args, device, rank):
    g = torch.Generator(device=device)
    g.manual_seed(1000 * rank + 7)
    real = torch.rand([args.batch_gpu, args.img_channels, args.res, args.res], generator=g, device=device) * 2 - 1
    lab = torch.randint(0, max(args.c_dim, 1), [args.batch_gpu], generator=g, device=device)
    real_c = torch.nn.functional.one_hot(lab, max(args.c_dim, 1)).float()[:, :args.c_dim].contiguous()
    return real, real_c


def one_step(tr, args, device, real, real_c):
    n_ph = len(tr.phases)
    z = torch.randn([n_ph, args.batch_gpu, 512], device=device)
    lab = torch.randint(0, max(args.c_dim, 1), [n_ph, args.batch_gpu], device=device)
    c = torch.nn.functional.one_hot(lab, max(args.c_dim, 1)).float()[..., :args.c_dim]
    tr.step([real], [real_c], [[z[i]] for i in range(n_ph)], [[c[i]] for i in range(n_ph)])


def _layer_launch(device, res, C, dtype, N=32):
    """One launch of the fused modulated 3x3 synthesis-layer conv (sg2_conv3x3: modulation in the operand
    staging, demod + noise + bias + lrelu + clamp epilogue) on [N, C, res, res] -> [N, C, res, res]."""
    from torch_utils.ops import conv2d_gradfix as cg
    x = torch.randn([N, C, res, res], device=device, dtype=dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn([C, C, 3, 3], device=device) / np.sqrt(C * 9)).to(dtype)
    wp = cg._pack_conv(w)
    s = torch.rand([N, C], device=device) + 0.5
    d = torch.rand([N, C], device=device) + 0.5
    noise = torch.randn([N, res, res], device=device, dtype=dtype)
    b = torch.zeros([C], device=device)

    def launch():
        cg.conv3x3_fused(x, wp, C, in_scale=s, out_scale=d, noise=noise, noise_gain=0.1, bias=b, act=1,
                         gain=float(np.sqrt(2)), clamp=256.0)
    for _ in range(3):
        launch()
    reps = 20
    stream = torch.cuda.current_stream(device)       # the stream sg2_conv3x3 is launched on
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    flops = 2.0 * N * C * C * 9 * res * res                             # 2 N Cout Cin 9 H W
    esz = x.element_size()
    byts = (2 * N * C * res * res + N * res * res + C * C * 9) * esz + (2 * N * C + C) * 4   # x, y, noise, w, s, d, b
    return ms, flops, byts


def _measured_traffic(key, kernel):
    """HBM bytes per launch of the roofline launch from the committed PMC passes (tools/pmc_traffic.py ->
    profiles/roofline_traffic.json), if they were taken on this exact launch configuration and kernel."""
    try:
        with open(os.path.join(ROOT, 'profiles', 'roofline_traffic.json')) as f:
            t = json.load(f)
        if t.get('config') != key or kernel not in t.get('kernel', ''):
            return None, None
        return t['hbm_bytes_per_launch'], t.get('hbm_bytes_per_launch_x2_rule')
    except (OSError, ValueError, KeyError):
        return None, None


def roofline(device, res, cbase, dtype, N=32):
    """Roofline of the dominant kernel, the LDS-halo MFMA 3x3 conv (sg2_conv3x3; at C = 64 its persistent
    form conv3x3_c64p_kernel), on the 256^2 synthesis layer the north star names.  Its
    arithmetic intensity (~286 FLOP/B at C = 64, 16-bit) is below the MI355X ridge (2500 TFLOP/s / 8 TB/s
    = 312 FLOP/B), so the bound is HBM: achieved = algorithmic bytes / measured launch time.  The MFMA
    view of the same launch and of the MFMA-bound 32^2 / C = 512 layer are reported beside it."""
    C = min(cbase // res, 512)
    ms, flops, byts = _layer_launch(device, res, C, dtype, N)
    ai = flops / byts
    ridge = MFMA_PEAK_FP16 * 1e12 / (HBM_PEAK * 1e9)
    key = f'sg2_conv3x3 fused {res}^2 C={C} N={N} {str(dtype).split(".")[-1]}'
    gbps = byts / (ms * 1e-3) / 1e9
    tflops = flops / (ms * 1e-3) / 1e12
    ring = C == 64 and os.environ.get('SG2_C64_RING', '1') != '0'
    kname = ('conv3x3_c64r_kernel (LDS-DMA halo ring, weights in registers)' if ring else
             'conv3x3_c64p_kernel (persistent, weights in LDS)') if C == 64 else 'conv3x3_halo_kernel'
    out = {'kernel': f'{kname} ({key}: modulation + demod/noise/bias/lrelu/clamp epilogue)'}
    if ai < ridge:
        out.update({'bound': 'hbm', 'achieved': round(gbps, 1), 'peak': HBM_PEAK, 'unit': 'GB/s',
                    'frac': round(gbps / HBM_PEAK, 4)})
    else:
        out.update({'bound': 'mfma', 'achieved': round(tflops, 2), 'peak': MFMA_PEAK_FP16, 'unit': 'TFLOP/s',
                    'frac': round(tflops / MFMA_PEAK_FP16, 4)})
    traffic, traffic_x2 = _measured_traffic(key, kname.split()[0] if C == 64 else 'conv3x3_halo_kernel')
    out.update({'traffic': traffic, 'traffic_fetch_x2_rule': traffic_x2, 'ms_per_launch': round(ms, 4),
                'algorithmic_flops_per_launch': flops, 'algorithmic_hbm_bytes_per_launch': byts,
                'arithmetic_intensity': round(ai, 1), 'ridge': round(ridge, 1),
                'mfma_tflops': round(tflops, 1), 'mfma_frac': round(tflops / MFMA_PEAK_FP16, 4)})
    ms2, fl2, _ = _layer_launch(device, 32, 512, dtype)
    out['mfma_bound_layer'] = {'kernel': 'conv3x3_halo_kernel, 32^2 C=512 N=32 (AI ~2300 FLOP/B)',
                               'ms_per_launch': round(ms2, 4), 'achieved': round(fl2 / (ms2 * 1e-3) / 1e12, 1),
                               'unit': 'TFLOP/s', 'frac': round(fl2 / (ms2 * 1e-3) / 1e12 / MFMA_PEAK_FP16, 4)}
    return out


def cpu_baseline(args):
    """CPU oracle (oracle/sg2_oracle.py, the reference's algorithm restated in PyTorch-CPU fp32) timed on
    the host cores: one Gmain, Greg, Dmain and Dreg phase at the bench resolution with batch 4
    (bounded sample), combined with the reference's phase frequencies (1, 1/4, 1, 1/16).  Beside it, the
    BASELINE configs[0] case (C1: the Claro yaml at 64^2 1-ch, batch 8, cbase 16384, map 8, c_dim 2), the
    reference's own CPU configuration, timed the same way at its full batch."""
    # the host cores this process may use: its CPU affinity, or the share the GPU box grants it
    # (OMP_NUM_THREADS; os.cpu_count() there reports the whole machine)
    threads = int(os.environ.get('OMP_NUM_THREADS') or len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
    out = _cpu_iteration(args.res, args.img_channels, args.c_dim, args.cbase, args.map_depth, 4, threads)
    c1 = _cpu_iteration(64, 1, 2, 16384, 8, 8, threads)
    c1['sample'] = 'BASELINE configs[0] (C1, claro_stylegan2-ada.yaml 64^2 1-ch bs8): ' + c1['sample']
    out['c1'] = c1
    return out


def _cpu_iteration(res, img_channels, c_dim, cbase, map_depth, B, threads):
    from oracle import sg2_oracle as O
    args = argparse.Namespace(res=res, img_channels=img_channels, c_dim=c_dim, cbase=cbase, map_depth=map_depth)
    torch.manual_seed(0)
    G = O.Generator(z_dim=512, c_dim=args.c_dim, w_dim=512, img_resolution=args.res, img_channels=args.img_channels,
                    channel_base=args.cbase, channel_max=512, num_fp16_res=4, conv_clamp=256,
                    fused_modconv_default='inference_only',
                    mapping_kwargs=dict(num_layers=args.map_depth)).train().requires_grad_(False)
    D = O.Discriminator(c_dim=args.c_dim, img_resolution=args.res, img_channels=args.img_channels,
                        channel_base=args.cbase, channel_max=512, num_fp16_res=4, conv_clamp=256,
                        epilogue_kwargs=dict(mbstd_group_size=4)).train().requires_grad_(False)
    aug = O.AugmentPipe(xflip=1, xint=1, scale=1, rotate=1, aniso=1, xfrac=1, xint_max=0.05, rotate_max=3 / 360,
                        xfrac_std=0.05, scale_std=0.05, aniso_std=0.05)
    aug.p.fill_(0.2)
    loss = O.StyleGAN2Loss(None, G, D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9, pl_weight=2)
    real = torch.rand([B, args.img_channels, args.res, args.res]) * 2 - 1
    c = torch.nn.functional.one_hot(torch.randint(0, max(args.c_dim, 1), [B]), max(args.c_dim, 1)).float()[:, :args.c_dim]
    t = {}
    for ph, mod, gain in [('Gmain', G, 1), ('Greg', G, 4), ('Dmain', D, 1), ('Dreg', D, 16)]:
        mod.requires_grad_(True)
        t0 = time.perf_counter()
        loss.accumulate_gradients(ph, real, c, torch.randn([B, 512]), c, gain, 0)
        t[ph] = time.perf_counter() - t0
        mod.requires_grad_(False)
        for p in mod.parameters():
            p.grad = None
    sec_per_iter = t['Gmain'] + t['Dmain'] + t['Greg'] / 4 + t['Dreg'] / 16
    return {'value': round(B / sec_per_iter, 4), 'unit': 'imgs/s', 'cores': threads, 'kind': 'port',
            'sample': f'oracle CPU fp32, {args.res}^2 {args.img_channels}-ch cbase {args.cbase}, batch {B}: one '
                      f'Gmain/Greg/Dmain/Dreg each ({", ".join(f"{k} {v:.1f}s" for k, v in t.items())}), '
                      f'combined at frequencies 1, 1/4, 1, 1/16; optimizer/EMA excluded'}


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    num_gpus = world
    # Rehearsal of the multi-rank path on a 1-GPU box (never the measured configuration):
    # SG2_BENCH_BACKEND=gloo SG2_BENCH_SHARE_DEVICE=1 puts every rank on cuda:0 and exchanges over gloo.
    backend = os.environ.get('SG2_BENCH_BACKEND', 'nccl')
    dev_index = 0 if os.environ.get('SG2_BENCH_SHARE_DEVICE') == '1' else local_rank
    if world > 1:
        torch.cuda.set_device(dev_index)
        if backend == 'nccl':
            torch.distributed.init_process_group('nccl', device_id=torch.device('cuda', dev_index))
        else:
            torch.distributed.init_process_group(backend)
    device = torch.device('cuda', dev_index)
    torch.backends.cudnn.benchmark = True

    tr = build(args, device, rank, num_gpus)
    real, real_c = make_inputs(args, device, rank)
    for _ in range(args.warmup):
        one_step(tr, args, device, real, real_c)
    graphs = args.graphs != 'off' and not args.no_graphs
    if graphs and args.graphs == 'auto' and num_gpus > 1:
        graphs = backend == 'nccl' and rccl_graph_ok(device, world)   # gloo cannot be captured
        if rank == 0:
            print(f'[bench] phase graphs at {world} ranks: {"on (RCCL capture probe passed)" if graphs else "off"}',
                  file=sys.stderr, flush=True)
    if graphs:
        # capture: one untimed step at batch_idx 0 runs (and captures) all four phases; afterwards every
        # phase is a single HIP-graph replay (trainer.py Trainer.graphs; with several GPUs the bucket
        # all_reduces are captured into the phase graphs)
        tr.graphs = True
        tr.batch_idx = 0
        one_step(tr, args, device, real, real_c)
    torch.cuda.synchronize(device)
    tr.batch_idx = 0                                    # timed region starts a full 16-step cycle
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step(tr, args, device, real, real_c)
    torch.cuda.synchronize(device)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t)

    imgs = args.steps * args.batch_gpu * num_gpus
    value = imgs / elapsed
    phase_ms = None
    if args.phase_timing:
        phase_ms = {ph.name: round(ph.start_event.elapsed_time(ph.end_event), 2) for ph in tr.phases
                    if ph.start_event is not None}
    roof = None
    if not args.no_roofline:
        roof = roofline(device, args.res, args.cbase, torch.float16 if args.fp16_dtype == 'fp16' else torch.bfloat16,
                        args.batch_gpu)
    cpu = None
    if rank == 0 and num_gpus == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    if rank == 0:
        line = {
            'metric': f'imgs/sec at {args.res}^2 bs{args.batch_gpu}/GPU StyleGAN2-ADA training (+ sec/kimg)',
            'value': round(value, 3), 'unit': 'imgs/s', 'n_gpus': num_gpus, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
            'graphs': graphs,
            'scaling': 'weak', 'vs_baseline': None,
            'dtype': f'{args.fp16_dtype}+fp32 ({args.fp16_dtype} at the 4 highest resolutions, fp32 below; f32 accumulate)',
            'data': 'synthetic (U(-1,1) reals resident in HBM, device-drawn z, random one-hot c; random-init weights)',
            'config': {'workload': f'StyleGAN2-ADA train iteration, {args.res}x{args.res} {args.img_channels}-ch, '
                                   f'c_dim {args.c_dim}, cbase {args.cbase}, map {args.map_depth}, '
                                   'Gmain+Dmain / Greg every 4 / Dreg every 16, ADA geometric p=0.2',
                       'global_batch': args.batch_gpu * num_gpus, 'batch_gpu': args.batch_gpu,
                       'resolution': args.res, 'parallelism': f'dp{num_gpus}'},
            'imgs_per_sec_per_gpu': round(value / num_gpus, 3),
            'sec_per_kimg': round(1000.0 / value, 3),
            'roofline': roof,
            'cpu_baseline': cpu,
        }
        # what torch.distributed actually initialised (a scaling run can be checked from the line alone), and
        # the gradient buckets each phase exchanges
        line['dist'] = {'backend': torch.distributed.get_backend() if world > 1 else None,
                        'world_size': torch.distributed.get_world_size() if world > 1 else 1,
                        'buckets': {ph.name: len(ph.exchange.buckets) for ph in tr.phases},
                        'bucket_mb': 32, 'overlapped': num_gpus > 1}
        if phase_ms is not None:
            line['last_phase_ms'] = phase_ms
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
