"""Training-iteration parity at BASELINE.json configuration widths (test infrastructure).

One full iteration (Gmain, Greg, Dmain, Dreg with the reference's gains, nan_to_num, lazy-reg Adam,
G_ema) runs on identical states (golden_init.init_state, keyed by parameter names), inputs and RNG
draws (rngtape.Tape) through
  * the product (HIP kernels, cuda:0, training/trainer.py Trainer),
  * the CPU oracle (oracle/sg2_oracle.py, fp32),
and is compared by `golden_init.summarize` (per-tensor L2 norm + 8 sampled entries) -- against the
reference-generated fixture (tests/golden/train_c1.npz, BASELINE configs[0]) or against the oracle run
in the same test (C2/C4/C5 widths, where a reference fixture would be too large to commit).

Error measures (all relative):
  * norm:    |‖a‖ - ‖b‖| / ‖b‖ per tensor;
  * samples: max_i |a_i - b_i| / rms(b) per tensor, rms = ‖b‖ / sqrt(numel) -- entry errors scaled
             by the tensor's typical magnitude, so near-zero entries do not blow the ratio up;
  * stats:   relative L2 of each reported loss vector (signs skipped: sign(0±eps) is rounding).
"""
import ast
import copy
import os

import numpy as np
import torch

from golden_init import init_state, summarize, unpack
from rngtape import Tape

CLARO_AUG = dict(xflip=1, xint=1, scale=1, rotate=1, aniso=1, xfrac=1, xint_max=0.05, rotate_max=3 / 360,
                 xfrac_std=0.05, scale_std=0.05, aniso_std=0.05)
PHASES = ['Gmain', 'Greg', 'Dmain', 'Dreg']


def _nets(mod, cfg, num_fp16_res, fp16_dtype=None, **extra):
    gk, dk = {}, {}
    if fp16_dtype is not None:
        gk['fp16_dtype'] = fp16_dtype
        dk['block_kwargs'] = dict(fp16_dtype=fp16_dtype)
    G = mod.Generator(z_dim=cfg['z_dim'], c_dim=cfg['c_dim'], w_dim=cfg['w_dim'], img_resolution=cfg['img_resolution'],
                      img_channels=cfg['img_channels'], channel_base=cfg['channel_base'],
                      channel_max=cfg['channel_max'], num_fp16_res=num_fp16_res, conv_clamp=256,
                      fused_modconv_default='inference_only', mapping_kwargs=dict(num_layers=cfg['map_depth']),
                      **gk).train().requires_grad_(False)
    D = mod.Discriminator(c_dim=cfg['c_dim'], img_resolution=cfg['img_resolution'], img_channels=cfg['img_channels'],
                          channel_base=cfg['channel_base'], channel_max=cfg['channel_max'], num_fp16_res=num_fp16_res,
                          conv_clamp=256, epilogue_kwargs=dict(mbstd_group_size=cfg['mbstd']),
                          **dk).train().requires_grad_(False)
    init_state(G, seed=1)
    init_state(D, seed=2)
    return G, D


def make_inputs(cfg, seed=31):
    r = np.random.RandomState(seed)
    B, c_dim = cfg['batch'], cfg['c_dim']
    z = r.standard_normal((B, cfg['z_dim'])).astype(np.float32)
    c = np.eye(max(c_dim, 1), dtype=np.float32)[r.randint(max(c_dim, 1), size=B)][:, :c_dim]
    real = r.uniform(-1, 1, (B, cfg['img_channels'], cfg['img_resolution'], cfg['img_resolution'])).astype(np.float32)
    gen_z = r.standard_normal((4, B, cfg['z_dim'])).astype(np.float32)
    gen_c = np.eye(max(c_dim, 1), dtype=np.float32)[r.randint(max(c_dim, 1), size=(4, B))][..., :c_dim]
    return dict(z=z, c=c, real=real, gen_z=gen_z, gen_c=gen_c)


def _perturb(t, rel, gen):
    """t * (1 + rel * u), u = +-1 per entry: an f32-rounding-sized nudge of a state or input."""
    u = torch.randint(0, 2, t.shape, generator=gen).to(t.dtype) * 2 - 1
    return t * (1 + rel * u)


def run_oracle(cfg, inp, tape, aug_p=0.3, perturb=0.0, isolated=False, perturb_seed=12345):
    """The CPU oracle's iteration; `tape` records (mode 'record') or replays its draws.  perturb > 0: every
    parameter, real image and latent is multiplied by (1 +- perturb) first (a fixed random sign per entry) --
    evaluated in float64 with perturb = 2^-24 this measures how far an f32-sized change of the state moves
    each result, i.e. the conditioning every f32 implementation inherits."""
    from oracle import sg2_oracle as O
    torch.manual_seed(0)
    G, D = _nets(O, cfg, 4)
    if perturb:
        gen = torch.Generator().manual_seed(perturb_seed)
        with torch.no_grad():
            for m in (G, D):
                for _, p in sorted(m.named_parameters()):
                    p.copy_(_perturb(p, perturb, gen))
        inp = {k: (_perturb(torch.from_numpy(np.asarray(v, np.float64)), perturb, gen).numpy()
                   if k in ('real', 'gen_z', 'z') else v) for k, v in inp.items()}
    G_ema = copy.deepcopy(G).eval()
    aug = O.AugmentPipe(**CLARO_AUG)
    aug.p.fill_(aug_p)
    stats = []
    loss = O.StyleGAN2Loss(None, G, D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9, pl_weight=2,
                           pl_no_weight_grad=True, report=lambda n, v: stats.append((n, v.detach().clone())))
    out = {}

    def on_grads(name, module):
        out.update(summarize({n: p.grad for n, p in module.named_parameters() if p.grad is not None},
                             f'grad/{name}'))

    T = lambda a: torch.from_numpy(np.array(a, dtype=np.float64)).to(O.REAL)  # noqa: E731 (f32-exact inputs; perturbed ones keep their f64 nudge)
    ctx = tape.record() if not tape.entries else tape.replay()
    with ctx:
        O.train_iteration(loss, O.make_phases(G, D), G, G_ema, T(inp['real']), T(inp['c']), T(inp['gen_z']),
                          T(inp['gen_c']), batch_idx=0, cur_nimg=1000, batch_size=cfg['batch'], on_grads=on_grads,
                          isolated=isolated)
    out['pl_mean'] = loss.pl_mean.detach().numpy()
    if isolated:
        return out, [(n, v.numpy()) for n, v in stats]
    out.update(summarize(dict(G.named_parameters()), 'G1'))
    out.update(summarize(dict(D.named_parameters()), 'D1'))
    out.update(summarize(dict(G_ema.named_parameters()), 'Gema1'))
    return out, [(n, v.numpy()) for n, v in stats]


def run_oracle_f64(cfg, inp, tape, aug_p=0.3, perturb=0.0, isolated=False, emu16=None, perturb_seed=12345):
    """The oracle evaluated in float64 on the same draws: the rounding-free answer that f32 results (the
    reference's and the product's alike) are judged against.  emu16 (torch.float16 / bfloat16): the reference's
    16-bit GPU iteration instead -- its num_fp16_res blocks with every tensor rounded where the reference's is
    (oracle.sg2_oracle.EMU16), float64 in between."""
    from oracle import sg2_oracle as O
    prev = (O.REAL, torch.get_default_dtype(), O.EMU16)
    O.REAL = torch.float64
    O.EMU16 = emu16
    torch.set_default_dtype(torch.float64)
    try:
        return run_oracle(cfg, inp, tape, aug_p, perturb, isolated, perturb_seed)
    finally:
        O.REAL, O.EMU16 = prev[0], prev[2]
        torch.set_default_dtype(prev[1])


def _isolated_phases(tr, G, D, real, c, gz, gc):
    """Each of the trainer's phases from the starting state (the phase-isolated fixtures): parameters and buffers
    restored before every phase, the phase's forward / backward and gradient exchange as Trainer.step runs them
    (eager), then the exchange's /N and nan_to_num, and no optimiser step."""
    from torch_utils import misc
    start = [{k: v.detach().clone() for k, v in m.state_dict().items()} for m in (G, D)]
    for pi, ph in enumerate(tr.phases):
        with torch.no_grad():
            for m, sd in zip((G, D), start):
                for k, v in m.state_dict().items():
                    v.copy_(sd[k])
        ph.opt.zero_grad(set_to_none=True)
        ph.module.requires_grad_(True)
        tr._accumulate(ph, [real], [c], [gz[pi]], [gc[pi]])
        ph.module.requires_grad_(False)
        ph.exchange.finish(ph.name, None)
        misc.nan_to_num(ph.exchange.flat, nan=0, posinf=1e5, neginf=-1e5, out=ph.exchange.flat)
        tr.on_grads(ph.name, ph.module)
        ph.exchange._reset()


def run_product(cfg, inp, tape, dev, fp16_dtype=None, aug_p=0.3, graphs=False, isolated=False, deterministic=True,
                f32_exact=False, grouped_affine=True, perturb=0.0, perturb_seed=0):
    """The product's iteration on `dev`.  fp16_dtype None: all-f32 (num_fp16_res=0, the reference's CPU
    arithmetic); else the reference's GPU default num_fp16_res=4 in that 16-bit type.  isolated: every phase
    from the starting state, no optimiser step (the *_iso fixtures); returns the gradients, pl_mean and stats.
    deterministic: the library's fixed-order reductions (sg2hip.deterministic) -- the result is a function of
    the inputs, so a bound is met or missed by the code, not by a run's atomic order.  f32_exact: the f32 layers
    on the f32-input MFMA kernels (SG2_F32_EXACT=1) instead of the split-bf16 products (the other f32
    arithmetic of the library); grouped_affine False: the synthesis affine layers one GEMM each
    (networks_stylegan2.grouped_affine), another evaluation order of the styles (diagnostics only).  perturb > 0:
    every parameter, real image and latent multiplied by (1 +- perturb) in f32 first (seeded signs; 2^-23 moves
    an entry by about one f32 ulp) -- a state equal within f32 rounding, i.e. another draw of the 16-bit
    rounding pattern (diagnostics: the product's own spread, tools/nudge16.py)."""
    import sg2hip
    from torch_utils.ops import conv2d_gradfix as cg
    from training import networks_stylegan2 as nets
    prev = (os.environ.get('SG2_F32_EXACT'), cg.presplit, nets.grouped_affine)
    nets.grouped_affine = grouped_affine
    if f32_exact:
        os.environ['SG2_F32_EXACT'] = '1'
        cg.presplit = False
    try:
        with sg2hip.deterministic(deterministic, device=dev):
            return _run_product(cfg, inp, tape, dev, fp16_dtype, aug_p, graphs, isolated, perturb, perturb_seed,
                                deterministic)
    finally:
        if prev[0] is None:
            os.environ.pop('SG2_F32_EXACT', None)
        else:
            os.environ['SG2_F32_EXACT'] = prev[0]
        cg.presplit = prev[1]
        nets.grouped_affine = prev[2]


def _run_product(cfg, inp, tape, dev, fp16_dtype, aug_p, graphs, isolated, perturb=0.0, perturb_seed=0,
                 deterministic=True):
    from training import networks_stylegan2 as net, augment_mi, loss as loss_mod, trainer as trainer_mod
    torch.manual_seed(0)
    G, D = _nets(net, cfg, 0 if fp16_dtype is None else 4, fp16_dtype)
    if perturb:     # the same signs, in the same order, as run_oracle's nudge (the state rounded to f32)
        gen = torch.Generator().manual_seed(perturb_seed)
        with torch.no_grad():
            for mod in (G, D):
                for _, p in sorted(mod.named_parameters()):
                    p.copy_(_perturb(p.detach().cpu().double(), perturb, gen).float())
        inp = {k: (_perturb(torch.from_numpy(np.asarray(v, np.float64)), perturb, gen).float().numpy()
                   if k in ('real', 'gen_z', 'z') else v) for k, v in inp.items()}
    G, D = G.to(dev), D.to(dev)
    G_ema = copy.deepcopy(G).eval()
    aug = augment_mi.AugmentPipe(run_dir=None, batch_size=cfg['batch'], **CLARO_AUG).train().requires_grad_(False).to(dev)
    aug.p.copy_(torch.as_tensor(aug_p))
    loss = loss_mod.StyleGAN2Loss(device=dev, G=G, D=D, augment_pipe=aug, r1_gamma=0.4096, style_mixing_prob=0.9,
                                  pl_weight=2, pl_no_weight_grad=True)
    opt = dict(class_name='torch.optim.Adam', lr=0.0025, betas=[0, 0.99], eps=1e-8)
    tr = trainer_mod.Trainer(G, D, G_ema, loss, opt, opt, batch_size=cfg['batch'], batch_gpu=cfg['batch'],
                             num_gpus=1, rank=0, device=dev, deterministic=deterministic)
    out, stats = {}, []

    def on_grads(name, module):
        out.update(summarize({n: p.grad for n, p in module.named_parameters() if p.grad is not None},
                             f'grad/{name}'))

    tr.on_grads = on_grads
    tr.cur_nimg = 1000
    orig = loss_mod.training_stats.report
    loss_mod.training_stats.report = lambda n, v: (stats.append((n, v.detach().float().cpu().numpy())), v)[1]
    T = lambda a: torch.from_numpy(np.array(a, dtype=np.float32)).to(dev)  # noqa: E731
    try:
        with tape.replay():
            gz, gc = T(inp['gen_z']), T(inp['gen_c'])
            if isolated:
                _isolated_phases(tr, G, D, T(inp['real']), T(inp['c']), gz, gc)
            else:
                tr.step([T(inp['real'])], [T(inp['c'])], [[gz[i]] for i in range(4)], [[gc[i]] for i in range(4)])
        torch.cuda.synchronize(dev)
    finally:
        loss_mod.training_stats.report = orig
    assert tape.pos == len(tape.entries), 'product consumed a different number of random draws'
    out['pl_mean'] = loss.pl_mean.detach().cpu().numpy()
    if isolated:
        return out, stats
    out.update(summarize(dict(G.named_parameters()), 'G1'))
    out.update(summarize(dict(D.named_parameters()), 'D1'))
    out.update(summarize(dict(G_ema.named_parameters()), 'Gema1'))
    return out, stats


def compare(got, want, tol_norm, tol_samples, groups=('grad/', 'G1/', 'D1/', 'Gema1/')):
    """Returns {group: (worst norm err, worst sample err, key)}; asserts key sets match."""
    keys_w, keys_g = _keys(want, groups), _keys(got, groups)
    _one_sided_zero(got, want, keys_g, keys_w)
    keys_w = sorted(set(keys_w) & set(keys_g))
    worst = {}
    for k in keys_w:
        nw, ng = float(want[k + '/norm']), float(got[k + '/norm'])
        sw, sg = np.asarray(want[k + '/samples'], np.float64), np.asarray(got[k + '/samples'], np.float64)
        if nw == 0:
            e_norm = 0.0 if ng == 0 else float('inf')
        else:
            e_norm = abs(ng - nw) / nw
        rms = max(nw / np.sqrt(float(want[k + '/numel'])), 1e-30)
        e_s = float(np.max(np.abs(sg - sw))) / rms if nw > 0 else float(np.max(np.abs(sg), initial=0.0))
        g = 'grad/' + k.split('/')[1] if k.startswith('grad/') else k.split('/')[0]
        w = worst.get(g, (0.0, 0.0, None))
        worst[g] = (max(w[0], e_norm), max(w[1], e_s), k if (e_norm > w[0] or e_s > w[1]) else w[2])
        assert e_norm <= tol_norm, f'{k}: norm rel err {e_norm:.3g} > {tol_norm}'
        assert e_s <= tol_samples, f'{k}: sampled-entry err {e_s:.3g} (x rms) > {tol_samples}'
    return worst


def _tensor_errs(a, b, k):
    """(norm error, sampled-entry error) of summary `a` against summary `b` for tensor key k."""
    nb, na = float(b[k + '/norm']), float(a[k + '/norm'])
    if nb == 0:
        return (0.0 if na == 0 else float('inf')), float(np.max(np.abs(np.asarray(a[k + '/samples'])), initial=0.0))
    rms = nb / np.sqrt(float(b[k + '/numel']))
    sa, sb = np.asarray(a[k + '/samples'], np.float64), np.asarray(b[k + '/samples'], np.float64)
    return abs(na - nb) / nb, float(np.max(np.abs(sa - sb), initial=0.0)) / rms


# (norm, sampled-entry) floors: gradients; parameters after the step -- Adam's first steps move an element by
# ~lr * sign(g), so a gradient element that is zero up to rounding (in the reference's f32 as much as here)
# may move the other way: one such element of a 512-bias (|p| ~ 0.1) shifts its norm by ~2e-4 and the
# element by ~0.05 of the tensor's rms.
F32_FLOORS = {'grad': (1e-4, 1e-3), 'param': (1e-3, 1e-1)}


def _group(k):
    return 'grad/' + k.split('/')[1] if k.startswith('grad/') else k.split('/')[0]


def _conditioning(fix):
    """The fixture's reference-derived f32 re-evaluations ('r32_<name>/', tests/golden/make_ref_spread.py): the
    REFERENCE's own f32 iteration run again with one thread (another oneDNN / MKL summation order) and at states
    nudged by (1 +- 2^-24) per entry (half an f32 ulp, several sign seeds).  How far each lands from the float64
    answer is the spread the reference's own f32 arithmetic has on that tensor -- discrete events included (C2 Greg:
    a half-ulp nudge moves the reference's b256.conv1.noise_strength gradient 18 % off float64).
    -> [(name, summary dict)]."""
    out = []
    for p in sorted({k.split('/', 1)[0] for k in fix if k.startswith('r32_')}):
        out.append((p, {k[len(p) + 1:]: v for k, v in fix.items() if k.startswith(p + '/')}))
    return out


GROUP_Q = 1.0     # the quantile of the phase's reference spreads the group term scales (1.0: the worst)


def judge_f32(got, fix, floors=F32_FLOORS, factor=4.0, group_factor=3.0,
              groups=('grad/', 'G1/', 'D1/', 'Gema1/'), check=True):
    """f32 results against the float64 answer (fixture keys 'f64/...'), per tensor k of group g (a phase's
    gradients, or a network after the step):

        err(got_k, f64) <= max(floor, factor * R_k, group_factor * max_{j in g} R_j),
        R_k = max(err(ref_k, f64), err(r32_<name>_k, f64) for every re-evaluation of the reference)

    i.e. the reference's own f32 spread on the tensor, from the fixture's reference run and the reference's
    re-evaluations (_conditioning) -- every term is the reference's arithmetic; nothing compares the product with
    itself.  Well-conditioned tensors are held to the floor (1e-4 on a gradient's norm).  Near-cancelling sums are
    not: the reference's own f32 results are off by up to percents there (noise-strength gradients, R1 bias
    gradients, tensors behind an lrelu mask that rounding flips).  Which tensor of a phase draws the short straw is
    chance, so the bound also admits the reference's worst spread in the same phase.

    Returns ({group: (worst norm err, worst sample err, worst reference norm err, worst ratio to the bound, its
    tensor)} plus worst['bound_terms'] = {term: number of tensors whose bound that term set} (floor / ref /
    r32_<name> / group), sorted ratios); raises after computing everything when `check` and any tensor is out of
    bounds."""
    truth = {k[4:]: v for k, v in fix.items() if k.startswith('f64/')}
    conds = _conditioning(fix)
    kw, kg = _keys(truth, groups), _keys(got, groups)
    _one_sided_zero(got, truth, kg, kw)
    keys = sorted(set(kw) & set(kg))
    errs, src = {}, {}
    for k in keys:
        rn, rs_ = _tensor_errs(fix, truth, k)
        sn = ss = 'ref'
        for name, cond in conds:
            if k + '/norm' in cond:
                cn, cs = _tensor_errs(cond, truth, k)
                if cn > rn:
                    rn, sn = cn, name
                if cs > rs_:
                    rs_, ss = cs, name
        errs[k] = (_tensor_errs(got, truth, k), (rn, rs_))
        src[k] = (sn, ss)
    per = {}
    for k, (_, (rn, rs_)) in errs.items():
        per.setdefault(_group(k), []).append((rn, rs_))
    gmax = {g: (float(np.quantile([v[0] for v in vs], GROUP_Q)), float(np.quantile([v[1] for v in vs], GROUP_Q)))
            for g, vs in per.items()}
    worst, ratios, fails, terms = {}, [], [], {}
    for k in keys:
        (gn, gs), (rn, rs_) = errs[k]
        g = _group(k)
        floor = floors['grad' if k.startswith('grad/') else 'param']
        cand_n = [(floor[0], 'floor'), (factor * rn, src[k][0]), (group_factor * gmax[g][0], 'group')]
        cand_s = [(floor[1], 'floor'), (factor * rs_, src[k][1]), (group_factor * gmax[g][1], 'group')]
        bn, tn = max(cand_n)
        bs, ts = max(cand_s)
        term = tn if gn / bn >= gs / bs else ts
        terms[term] = terms.get(term, 0) + 1
        w = worst.get(g, (0.0, 0.0, 0.0, 0.0, ''))
        ratio = max(gn / bn, gs / bs)
        ratios.append(ratio)
        worst[g] = (max(w[0], gn), max(w[1], gs), max(w[2], rn), max(w[3], ratio), k if ratio > w[3] else w[4])
        if gn > bn:
            fails.append(f'{k}: norm err vs f64 {gn:.3g} > bound {bn:.3g} (set by {tn}; reference spread {rn:.3g}, phase max {gmax[g][0]:.3g})')
        if gs > bs:
            fails.append(f'{k}: sampled-entry err vs f64 {gs:.3g} > bound {bs:.3g} (set by {ts}; reference spread {rs_:.3g})')
    worst['bound_terms'] = terms
    if check:
        assert not fails, f'{len(fails)} tensors out of bounds; first: {fails[0]}'
    return worst, sorted(ratios)


def judge_vs_reference(got, fix, well=1e-4, tol=3e-4, factor=4.0, groups=('grad/',), check=True):
    """Direct product-vs-reference-f32 check on every tensor the reference's f32 result gets right (both its
    norm and its sampled entries within `well` of the float64 answer, in its run and every re-evaluation): the
    product must then agree with the reference itself to max(tol, (factor + 1) x R) on each measure, R the
    reference's spread on that measure (judge_f32's R_k) -- the triangle bound of judge_f32's per-tensor
    allowance (factor x R from float64) plus the reference's own distance from float64; measured: C4 Gmain
    b256.torgb.affine.bias, whose reference re-evaluations spread its sampled entries by 9.7e-5 of the rms.
    Scalar parameters (the noise strengths) are left to judge_f32: each gradient is ONE reduction over every pixel
    of the layer, near-cancelling, whose f32 value moves with the summation order (measured: C1 Greg
    b64.conv1.noise_strength, float-atomic mode, 3.0e-4 from float64 in one run and within 1e-4 in another; the
    reference's re-evaluations keep its own order and spread 5.5e-5), which the reference's spread does not sample.  Gradients only: a parameter after Adam's first step (beta1 = 0) moves each entry by
    about lr * sign(g), so an entry whose gradient is zero up to rounding lands 2 lr apart in two correct
    evaluations (measured: D1/b512.conv1.bias at C4 / p = 0); the parameters are held by the flat check.
    Returns (number of tensors checked, worst ratio to the bound, its key)."""
    truth = {k[4:]: v for k, v in fix.items() if k.startswith('f64/')}
    conds = _conditioning(fix)
    keys = sorted(set(_keys(truth, groups)) & set(_keys(got, groups)))
    n, worst, wk, fails = 0, 0.0, '', []
    for k in keys:
        rn, rs_ = _tensor_errs(fix, truth, k)
        for _, c in conds:
            if k + '/norm' in c:
                cn, cs = _tensor_errs(c, truth, k)
                rn, rs_ = max(rn, cn), max(rs_, cs)
        if max(rn, rs_) >= well or float(fix[k + '/norm']) == 0.0 or int(fix[k + '/numel']) == 1:
            continue
        n += 1
        en, es = _tensor_errs(got, fix, k)
        tn, ts = max(tol, (factor + 1) * rn), max(tol, (factor + 1) * rs_)
        if max(en / tn, es / ts) > worst:
            worst, wk = max(en / tn, es / ts), k
        if en > tn or es > ts:
            fails.append(f'{k}: vs reference f32 norm {en:.3g} (bound {tn:.3g}) samples {es:.3g} (bound {ts:.3g})')
    if check:
        assert not fails, f'{len(fails)} of {n} well-conditioned tensors differ from the reference: {fails[0]}'
    return n, worst, wk


def judge_flat(got_flat, ref_flat, floor, factor=3.0):
    """Per group: the estimated whole-vector error vs f64 (compare_flat) within max(floor, factor x the
    reference f32's).  `floor` is one number or (norm-vector floor, sampled-entry floor)."""
    fn, fs = floor if isinstance(floor, tuple) else (floor, floor)
    for g, (en, es) in got_flat.items():
        tn = max(fn, factor * max(ref_flat[g]))
        ts = max(fs, factor * max(ref_flat[g]))
        assert en <= tn and es <= ts, f'{g}: norm-vector err {en:.3g} (bound {tn:.3g}), flat err {es:.3g} (bound {ts:.3g})'


# The regulariser statistics inherit the conditioning of the gradients they are built from: J^T y of the
# path-length pass carries ~7e-4 of inherent f32 error (the oracle's own f32 vs float64 at C2), and the
# penalty squares (|J^T y| - a).
REG_STATS = ('Loss/pl_penalty', 'Loss/G/reg', 'Loss/r1_penalty', 'Loss/D/reg')


def judge_stats_f32(got, fix, floor=1e-4, reg_floor=3e-3, factor=4.0, group_factor=3.0, check=True):
    """Reported loss statistics against f64: each within max(floor, factor x the reference f32's error on it,
    group_factor x the reference's worst statistic error) -- the same chance argument as judge_f32."""
    names, ref_vals = fixture_stats(fix)
    assert [n for n, _ in got] == names, 'reported statistics differ in name or order'
    rows = []
    for j, ((n, v), r) in enumerate(zip(got, ref_vals)):
        if 'signs' in n:
            continue
        t = np.asarray(fix[f'f64/stats/{j}'], np.float64)
        den = max(np.linalg.norm(t), 1e-30)
        rows.append((n, np.linalg.norm(np.asarray(v, np.float64) - t) / den,
                     np.linalg.norm(np.asarray(r, np.float64) - t) / den))
    gmax = max(er for _, _, er in rows)
    for n, e, er in rows:
        fl = reg_floor if n in REG_STATS else floor
        t = max(fl, factor * er, group_factor * gmax)
        assert not check or e <= t, \
            f'stat {n}: rel err vs f64 {e:.3g} > bound {t:.3g} (reference f32 {er:.3g}, worst reference stat {gmax:.3g})'
    return max(e for _, e, _ in rows)


def judge_pl_mean(got, fix, floor=3e-3, factor=4.0, check=True):
    t = float(fix['f64/pl_mean'])
    e = abs(float(got['pl_mean']) - t) / abs(t)
    er = abs(float(fix['pl_mean']) - t) / abs(t)
    assert not check or e <= max(floor, factor * er), f'pl_mean rel err vs f64 {e:.3g} (reference f32 {er:.3g})'
    return e


def _keys(d, groups):
    return sorted(k[:-5] for k in d if k.endswith('/norm') and k.startswith(tuple(groups)))


def _one_sided_zero(got, want, keys_g, keys_w):
    """A parameter whose gradient is structurally zero (e.g. a toRGB bias in the path-length pass) may be
    materialised as zeros on one side and absent on the other -- the reference's own CUDA and CPU paths
    differ there.  Anything else must be present on both sides."""
    for k in sorted(set(keys_g) ^ set(keys_w)):
        d = got if k in keys_g else want
        assert float(d[k + '/norm']) == 0.0, f'{k} present on one side only with norm {float(d[k + "/norm"]):.3g}'


def compare_stats(got, want_names, want_vals, tol):
    assert [n for n, _ in got] == list(want_names), 'reported statistics differ in name or order'
    worst = 0.0
    for (n, v), w in zip(got, want_vals):
        if 'signs' in n:
            continue
        v, w = np.asarray(v, np.float64), np.asarray(w, np.float64)
        e = np.linalg.norm(v - w) / max(np.linalg.norm(w), 1e-30)
        worst = max(worst, e)
        assert e <= tol, f'stat {n}: rel err {e:.3g} > {tol}'
    return worst


def fixture_stats(z):
    names, vals = [], []
    for ph in PHASES:
        nm = [str(s) for s in z[f'stats_names/{ph}']]
        names += nm
        vals += [z[f'stats/{ph}/{j}'] for j in range(len(nm))]
    return names, vals


def load_fixture(npz):
    """-> (cfg, inputs, tape, fixture dict with the summaries unpacked)"""
    z = unpack(npz)
    cfg = ast.literal_eval(str(z['cfg']))
    return cfg, make_inputs(cfg, cfg['input_seed']), Tape.from_npz(z, 'tape'), z


def compare_flat(got, want, groups):
    """Mixed-precision measure, per group (a phase's gradients, or a network's parameters):
      * the relative L2 error of the vector of tensor norms;
      * the relative L2 error of the group's whole flat vector, estimated from the sampled entries:
        sqrt(sum_i numel_i * mean_s (a_s - b_s)^2) / sqrt(sum_i |b_i|^2) -- the measure of a flat
        concatenated gradient (the vector the all-reduce exchanges), weighting tensors by their size."""
    res = {}
    for g in groups:
        kw, kg = _keys(want, [g + '/']), _keys(got, [g + '/'])
        _one_sided_zero(got, want, kg, kw)
        keys = sorted(set(kw) & set(kg))
        assert keys, g
        na = np.array([float(got[k + '/norm']) for k in keys])
        nb = np.array([float(want[k + '/norm']) for k in keys])
        err2 = sum(float(want[k + '/numel']) * float(np.mean((np.asarray(got[k + '/samples'], np.float64) -
                                                               np.asarray(want[k + '/samples'], np.float64)) ** 2))
                   for k in keys)
        res[g] = (float(np.linalg.norm(na - nb) / np.linalg.norm(nb)), float(np.sqrt(err2) / np.linalg.norm(nb)))
    return res


def reference_flat(fix, truth, groups):
    """compare_flat of the reference's f32 evaluations (the fixture's run and each re-evaluation, _conditioning):
    per group the largest of each measure -- the reference's own f32 spread on the phase's flat vector."""
    out = compare_flat(fix, truth, groups)
    for _, cond in _conditioning(fix):
        c = compare_flat(cond, truth, groups)
        out = {g: (max(out[g][0], c[g][0]), max(out[g][1], c[g][1])) for g in out}
    return out


def save_summary(tag, got):
    """Keep the product's summaries next to the measured errors (gpurun_out/summ_<tag>.npz)."""
    import os
    from golden_init import pack
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out')
    os.makedirs(d, exist_ok=True)
    np.savez_compressed(os.path.join(d, f'summ_{tag}.npz'), **pack({k: v for k, v in got.items()}))


def record(tag, data):
    """Append measured errors to gpurun_out/config_parity.jsonl (evidence for the tolerances)."""
    import json
    import os
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out')
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, 'config_parity.jsonl'), 'a') as f:
        f.write(json.dumps({'tag': tag, **{k: v for k, v in data.items()}}, default=str) + '\n')
