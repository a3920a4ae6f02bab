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
K = 16 is exactly one cycle (4 Greg, 1 Dreg); the default K = 112 is seven whole cycles (>= 100 timed
iterations covering whole 16-iteration cycles, ~5 s timed).  A K that is not a multiple of 16 carries a partial cycle:
K = 20 has 5 Greg and 2 Dreg (10 % Dreg steps against the schedule's 6.25 %, so a 20-step value is slightly
pessimistic).
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
    ap.add_argument('--steps', type=int, default=112)
    ap.add_argument('--warmup', type=int, default=8)
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
    ap.add_argument('--deterministic', default='on', choices=['on', 'off'],
                    help='the training iteration\'s reductions: the library\'s fixed-order slots (on, the default: '
                         'Trainer(deterministic=True)) or float atomics (off, an A/B mode)')
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
                             phase_timing=args.phase_timing, deterministic=args.deterministic == 'on')
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
    ring = C == 64 and os.environ.get('SG2_C64_RING', '49') != '0'
    ring32 = C == 32 and os.environ.get('SG2_C32_RING', '1') != '0'
    kname = ('conv3x3_c64r_kernel (LDS-DMA halo ring, weights in registers)' if ring else
             'conv3x3_c64p_kernel (persistent, weights in LDS)') if C == 64 else (
        'conv3x3_c32r_kernel (LDS-DMA halo ring, 32 x 8 tiles, weights in registers)' if ring32 else
        'conv3x3_halo_kernel')
    out = {'kernel': f'{kname} ({key}: modulation + demod/noise/bias/lrelu/clamp epilogue)'}
    if ai < ridge:
        out.update({'bound': 'hbm', 'achieved': round(gbps, 1), 'peak': HBM_PEAK, 'unit': 'GB/s',
                    'frac': round(gbps / HBM_PEAK, 4)})
    else:
        out.update({'bound': 'mfma', 'achieved': round(tflops, 2), 'peak': MFMA_PEAK_FP16, 'unit': 'TFLOP/s',
                    'frac': round(tflops / MFMA_PEAK_FP16, 4)})
    traffic, traffic_x2 = _measured_traffic(key, kname.split()[0])
    out.update({'traffic': traffic, 'traffic_fetch_x2_rule': traffic_x2, 'ms_per_launch': round(ms, 4),
                'algorithmic_flops_per_launch': flops, 'algorithmic_hbm_bytes_per_launch': byts,
                'arithmetic_intensity': round(ai, 1), 'ridge': round(ridge, 1),
                'mfma_tflops': round(tflops, 1), 'mfma_frac': round(tflops / MFMA_PEAK_FP16, 4)})
    ms2, fl2, _ = _layer_launch(device, 32, 512, dtype)
    out['mfma_bound_layer'] = {'kernel': 'conv3x3_halo_kernel, 32^2 C=512 N=32 (AI ~2300 FLOP/B)',
                               'ms_per_launch': round(ms2, 4), 'achieved': round(fl2 / (ms2 * 1e-3) / 1e12, 1),
                               'unit': 'TFLOP/s', 'frac': round(fl2 / (ms2 * 1e-3) / 1e12 / MFMA_PEAK_FP16, 4)}
    return out


def exchange_diagnostics(tr, args, device, real, real_c, world):
    """After the timed region, at N > 1: one eager 16-step cycle with HIP events per phase (Trainer.exchange_timing)
    -> per phase the flat gradient bytes all-reduced, the bucket count, the forward + backward time and the exposed
    exchange time (backward issued -> every bucket's all_reduce complete, on the compute stream): what the
    bucketed, hook-overlapped RCCL exchange did not hide behind the backward (reference exchange:
    training_loop_mi_multimodal.py:341-351).  Also a standalone all_reduce of each module's flat buffer (the
    unhidden cost for comparison)."""
    graphs = tr.graphs
    tr.graphs = False
    tr.exchange_timing = {}
    tr.batch_idx = 0
    for _ in range(16):
        one_step(tr, args, device, real, real_c)
    torch.cuda.synchronize(device)
    res = {}
    for ph in tr.phases:
        evs = tr.exchange_timing.get(ph.name, [])
        if not evs:
            continue
        fb = [a.elapsed_time(b) for a, b, _ in evs]
        ex = [b.elapsed_time(c) for _, b, c in evs]
        res[ph.name] = {'allreduce_bytes': int(ph.exchange.total * 4), 'buckets': len(ph.exchange.buckets),
                        'fwd_bwd_ms': round(float(np.mean(fb)), 3), 'exposed_exchange_ms': round(float(np.mean(ex)), 3),
                        'steps': len(evs)}
    for name, ph in (('G', tr.phases[0]), ('D', tr.phases[-1])):
        flat = ph.exchange.flat
        if flat is None:
            continue
        buf = flat.clone()
        res[f'standalone_allreduce_{name}_ms'] = round(_time_ms(lambda: torch.distributed.all_reduce(buf), reps=5), 3)
    tr.exchange_timing = None
    tr.graphs = graphs
    return res


def _time_ms(fn, reps=20):
    """Average ms per call of fn (one or more launches on the current stream) with HIP events on that stream."""
    for _ in range(3):
        fn()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def _roof_entry(kernel, shape, ms, flops, byts, mfma_peak=None):
    """One family's roofline: the binding roof of the launch is min(MFMA peak, AI x HBM peak); frac = achieved rate
    / that roof, in the roof's unit.  mfma_peak: the compute roof in TFLOP/s when it is not the dense 16-bit one."""
    mfma_peak = mfma_peak or MFMA_PEAK_FP16
    ai = flops / byts if byts else float('inf')
    tfl = flops / (ms * 1e-3) / 1e12
    gbps = byts / (ms * 1e-3) / 1e9
    hbm_bound = ai * HBM_PEAK * 1e9 < mfma_peak * 1e12
    e = {'kernel': kernel, 'shape': shape, 'ms_per_launch': round(ms, 4), 'algorithmic_flops_per_launch': flops,
         'algorithmic_hbm_bytes_per_launch': byts, 'arithmetic_intensity': round(ai, 1)}
    if hbm_bound:
        e.update({'bound': 'hbm', 'achieved': round(gbps, 1), 'peak': HBM_PEAK, 'unit': 'GB/s',
                  'frac': round(gbps / HBM_PEAK, 4)})
    else:
        e.update({'bound': 'mfma', 'achieved': round(tfl, 1), 'peak': round(mfma_peak, 1), 'unit': 'TFLOP/s',
                  'frac': round(tfl / mfma_peak, 4)})
    if flops:
        e['mfma_tflops'] = round(tfl, 1)
    return e


def roofline_families(device, dtype=torch.float16):
    """Rooflines of the kernel families that dominate the 256^2 step (profiles/r0*_step_breakdown.txt), each on its
    largest launch of the bench workload, timed with HIP events on the launching stream.  Algorithmic cost per
    launch: a conv 2 N Cout Cin taps OH OW FLOP and its input + output bytes (weights negligible); the FIR and the
    fused layer backward their input + output bytes (no FLOP counted: VALU work far under the HBM roof)."""
    from torch_utils.ops import conv2d_gradfix as cg, upfirdn2d
    import sg2hip
    esz = torch.tensor([], dtype=dtype).element_size()
    cl = torch.channels_last
    out = {}

    def rnd(*shape):
        return torch.randn(shape, device=device, dtype=dtype).contiguous(memory_format=cl)

    # the D down-2 conv of the 256^2 block after its FIR (Dmain batch 64) on its production route, the stride-2
    # LDS-DMA implicit GEMM (conv3x3_s2g_kernel; the generic implicit GEMM before round 5)
    N, Ci, H, Co = 64, 64, 257, 128
    OH = (H - 3) // 2 + 1
    x = rnd(N, Ci, H, H)
    wp = cg._pack_conv((torch.randn(Co, Ci, 3, 3, device=device) / 24).to(dtype))
    b = torch.zeros(Co, device=device)
    ms = _time_ms(lambda: cg.conv3x3_fused(x, wp, Co, bias=b, act=1, gain=1.41, clamp=256.0, stride=2))
    out['d_down_s2g'] = _roof_entry('conv3x3_s2g_kernel (stride-2 LDS-DMA implicit GEMM)',
                                    f'D down-2 3x3 N{N} {Ci}x{H}^2 -> {Co}x{OH}^2, bias + lrelu', ms,
                                    2.0 * N * Co * Ci * 9 * OH * OH, (N * Ci * H * H + N * Co * OH * OH) * esz)
    del x
    # up-2 transposed conv (conv3x3_up2_kernel, edge split) on the 32^2 -> 65^2 layer of the 64^2 synthesis block
    # (G forward, modulated): the generic implicit GEMM's largest 16-bit launch until the edge split moved it
    N, Ci, H, Co = 32, 512, 32, 256
    x = rnd(N, Ci, H, H)
    wp = cg._pack_conv((torch.randn(Co, Ci, 3, 3, device=device) / 68).to(dtype))
    s_ = torch.rand(N, Ci, device=device) + 0.5
    OT = 2 * H + 1
    assert cg._up2_ok(x, Co, OT, OT, 3, 3, 2, (0, 0), True)
    ms = _time_ms(lambda: cg.conv_fused(x, wp, Co, OT, OT, 3, 3, 2, (0, 0), transpose=True, in_scale=s_))
    out['up2_conv'] = _roof_entry('conv3x3_up2_kernel (cell tiles + edge strips)',
                                  f'up-2 transposed 3x3 N{N} {Ci}x{H}^2 -> {Co}x{OT}^2 (modulated)', ms,
                                  2.0 * N * Co * Ci * 9 * H * H, (N * Ci * H * H + N * Co * OT * OT) * esz)
    del x
    # generic implicit GEMM in f32 (conv_fwd_kernel, three-way bf16 split): its largest launch, the 16^2 C = 512
    # synthesis layer (bs32, modulated, bias + lrelu).  The split issues six bf16 products per f32 product, so its
    # compute roof is the dense 16-bit MFMA peak / 6 (the exact-f32 MFMA, v_mfma_f32_16x16x4_f32, peaks at 157.3)
    N, C, R = 32, 512, 16
    x = torch.randn(N, C, R, R, device=device).contiguous(memory_format=cl)
    wp = cg._pack_conv(torch.randn(C, C, 3, 3, device=device) / 68)
    s_ = torch.rand(N, C, device=device) + 0.5
    b = torch.zeros(C, device=device)
    ms = _time_ms(lambda: cg.conv_fused(x, wp, C, R, R, 3, 3, 1, (1, 1), in_scale=s_, out_scale=s_, bias=b, act=1,
                                        gain=1.41, clamp=256.0))
    out['conv_f32_split'] = _roof_entry('conv_fwd_kernel<float> (implicit GEMM, 3-way bf16 split)',
                                        f'3x3 s1 N{N} C{C} {R}^2 f32 (modulated, bias + lrelu)', ms,
                                        2.0 * N * C * C * 9 * R * R, 2 * N * C * R * R * 4,
                                        mfma_peak=MFMA_PEAK_FP16 / 6)
    del x
    # halo conv: the 128^2 C=128 synthesis layer (G forward, bs32)
    N, C, R = 32, 128, 128
    x = rnd(N, C, R, R)
    wp = cg._pack_conv((torch.randn(C, C, 3, 3, device=device) / 34).to(dtype))
    s_ = torch.rand(N, C, device=device) + 0.5
    ms = _time_ms(lambda: cg.conv3x3_fused(x, wp, C, in_scale=s_, out_scale=s_, bias=torch.zeros(C, device=device),
                                           act=1, gain=1.41, clamp=256.0))
    out['halo_conv'] = _roof_entry('conv3x3_halo_kernel', f'3x3 s1 N{N} C{C} {R}^2 (modulated, fused epilogue)', ms,
                                   2.0 * N * C * C * 9 * R * R, 2 * N * C * R * R * esz)
    # halo weight gradient at the same shape
    g = rnd(N, C, R, R)
    ms = _time_ms(lambda: cg._wgrad_raw(g, x, 3, 3, 1, (1, 1)))
    out['halo_wgrad'] = _roof_entry('wgrad3x3 (LDS-DMA halo)', f'3x3 s1 N{N} C{C}x{C} {R}^2', ms,
                                    2.0 * N * C * C * 9 * R * R, 2 * N * C * R * R * esz)
    del x, g
    # fused synthesis-layer first-order backward (sg2_layer_bwd) on the 256^2 C=64 layer
    N, C, R = 32, 64, 256
    dy, y, c = rnd(N, C, R, R), rnd(N, C, R, R), rnd(N, C, R, R)
    dc = torch.empty_like(dy)
    d = torch.rand(N, C, device=device) + 0.5
    db, dd = torch.zeros(C, device=device), torch.zeros(N, C, device=device)
    dn = torch.zeros(N, R, R, device=device)
    lib = sg2hip.lib()

    def lbwd():
        sg2hip.check(lib.sg2_layer_bwd(sg2hip.ptr(dc), sg2hip.ptr(db), sg2hip.ptr(dd), sg2hip.ptr(dn), sg2hip.ptr(dy),
                                       sg2hip.ptr(y), sg2hip.ptr(c), sg2hip.ptr(d), sg2hip.dtype_code(dy), N, R * R, C, 1, 0.2,
                                       1.41, 256.0, sg2hip.stream_ptr(device)), 'sg2_layer_bwd')
    ms = _time_ms(lbwd)
    out['layer_bwd'] = _roof_entry('layer_bwd_kernel', f'N{N} C{C} {R}^2: dy, y, c in; dc out (+ db, dd, dnoise)', ms,
                                   0, 4 * N * C * R * R * esz)
    del dy, y, c, dc
    # 4x4 FIR, up 1 / down 1 (upfirdn_nhwc_f4s): the D 256^2 pad-FIR before the down-2 conv (256^2 -> 257^2)
    x = rnd(64, 64, 256, 256)
    f = upfirdn2d.setup_filter([1, 3, 3, 1], device=device)
    ms = _time_ms(lambda: upfirdn2d.upfirdn2d(x, f, padding=2))
    out['fir_f4s'] = _roof_entry('upfirdn_nhwc_f4s', 'N64 C64 256^2 -> 257^2 (pad 2)', ms, 0,
                                 (64 * 64 * 256 * 256 + 64 * 64 * 257 * 257) * esz)
    del x
    weakest = min(out, key=lambda k: out[k]['frac'])
    out['weakest'] = weakest
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

    exch = None
    if world > 1:
        exch = exchange_diagnostics(tr, args, device, real, real_c, world)
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
    fams = None
    if not args.no_roofline and args.res == 256:
        fams = roofline_families(device, torch.float16 if args.fp16_dtype == 'fp16' else torch.bfloat16)
    cpu = None
    if rank == 0 and num_gpus == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    if rank == 0:
        line = {
            'metric': f'imgs/sec at {args.res}^2 bs{args.batch_gpu}/GPU StyleGAN2-ADA training (+ sec/kimg)',
            'value': round(value, 3), 'unit': 'imgs/s', 'n_gpus': num_gpus, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
            'graphs': graphs, 'deterministic': args.deterministic == 'on',
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
            'roofline_families': fams,
            'cpu_baseline': cpu,
        }
        # what torch.distributed actually initialised (a scaling run can be checked from the line alone), and
        # the gradient buckets each phase exchanges
        line['dist'] = {'backend': torch.distributed.get_backend() if world > 1 else None,
                        'world_size': torch.distributed.get_world_size() if world > 1 else 1,
                        'buckets': {ph.name: len(ph.exchange.buckets) for ph in tr.phases},
                        'bucket_mb': 32, 'overlapped': num_gpus > 1}
        if exch is not None:
            line['dist']['exchange'] = exch
        if phase_ms is not None:
            line['last_phase_ms'] = phase_ms
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
