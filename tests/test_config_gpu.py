"""Whole-iteration parity at every BASELINE.json configuration's real width, on the GPU, against
fixtures the REFERENCE generated (tests/golden/make_golden.py: the reference's fp32 CPU iteration and the
oracle's float64 evaluation of the same state, inputs and random draws):

  configs[0]    C1  train_c1.npz  64^2 1-ch bs8, cbase 16384, map 8, c_dim 2 (the Claro yaml)
  configs[1..2] C2  train_c2.npz  256^2 1-ch, cbase 16384, map 8, c_dim 2, batch 4 of 32
                                  (the DP exchange of configs[2]: tests/test_dist_gloo.py)
  configs[3]    C4  train_c4.npz  512^2 3-ch, cbase 32768, PL + R1, batch 2 of 16
  configs[4]    C5  train_c5.npz  1024^2 3-ch, cbase 32768, ADA, batch 2 of 8
plus full-batch runs of C4 (bs16, fp16) and C5 (bs8, bf16): every statistic / norm finite.

f32 product (num_fp16_res=0: the reference's CPU arithmetic), against the float64 answer: per tensor
within max(1e-4, 4 x the reference's own f32 error on it, 5 x the reference's worst error in the same
phase; see F32_GROUP_FACTOR) (config_parity.judge_f32), and per phase / network the whole-vector error within 3 x the
reference's (floor 1e-4 for gradients, 1e-5 for parameters).
16-bit product (num_fp16_res=4, the reference's GPU default, float16 or bfloat16 with f32 accumulate):
per phase / network, the relative error of the flat vector against the float64 answer
(config_parity.compare_flat), tolerances set from the measured errors (profiles/r02_config_parity.jsonl).
"""
import numpy as np
import pytest
import torch

from golden_util import load
import config_parity as cp

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)
GROUPS = ['grad/Gmain', 'grad/Greg', 'grad/Dmain', 'grad/Dreg', 'G1', 'D1', 'Gema1']

# 16-bit storage, f32 accumulate: per-group flat relative error vs the float64 answer must stay below
# max(floor, 2 x the reference's own f32 error on that group) -- the reference's f32 CPU result is itself
# off by up to 9% (C2 Dreg) / 16% (C5 Dreg) there.  Floors: the measured 16-bit errors
# (profiles/r02_config_parity.jsonl) with ~1.5x margin.  The regularisation phases are the noisy ones:
# the product's float atomics make repeated runs differ, and at C2 fp16 six runs gave Greg flat errors of
# 0.055-0.093 and Dreg 0.066-0.16 (profiles/r02_c2_fp16_repeats.jsonl), so their floors are 1.5x the
# largest of those.  The bf16 Gmain floor was 0.06 against a single measured 0.057 (C5): the round-3 ring conv
# rounds the modulated weight round(W * round(s)) where the reference rounds the modulated activation (one
# rounding either way) and measured 0.061 (0.057 with the ring off), so it takes the
# policy's 1.5x of the round-2 measurement, 0.085.
FLOOR16 = {
    'fp16': {'grad/Gmain': 0.03, 'grad/Greg': 0.14, 'grad/Dmain': 0.05, 'grad/Dreg': 0.24, 'param': 1e-3},
    'bf16': {'grad/Gmain': 0.085, 'grad/Greg': 0.2, 'grad/Dmain': 0.06, 'grad/Dreg': 0.15, 'param': 2e-3},
}


def _truth(fix):
    return {k[4:]: v for k, v in fix.items() if k.startswith('f64/')}


def _check_flat(res, ref, floors):
    for g, (en, es) in res.items():
        t = max(floors.get(g, floors['param']), 2 * max(ref[g]))
        assert en <= t and es <= t, f'{g}: norm-vector err {en:.3g}, flat err {es:.3g} (tol {t:.3g})'


F32_FACTOR = 4.0
# The product is not bitwise deterministic: split-K convolutions and the dot / bias / noise reductions
# accumulate with float atomics, so two runs on the same inputs differ (1130 of 1873 summary entries at C4,
# profiles/r02_f32_repeat_c4.log, tools/f32_repeat.py).  On the near-cancelling scalars (a layer's
# noise_strength gradient: a sum over N*H*W of dnoise * noise) the spread alone was 1.4x between two runs,
# so the per-phase term of the bound is 5 x the reference's worst error in the phase, not 3 x.
F32_GROUP_FACTOR = 5.0


@pytest.mark.timeout(240)
@pytest.mark.parametrize('tag', ['c1', 'c2', 'c4', 'c5'])
def test_f32_iteration_vs_reference(tag):
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}.npz'))
    got, stats = cp.run_product(cfg, inp, tape, DEV)
    cp.save_summary(f'{tag}_f32', got)
    worst, ratios = cp.judge_f32(got, fix, factor=F32_FACTOR, group_factor=F32_GROUP_FACTOR, check=False)
    ws = cp.judge_stats_f32(stats, fix, check=False)
    pl = cp.judge_pl_mean(got, fix, check=False)
    ref_flat = cp.compare_flat(fix, _truth(fix), GROUPS)
    flat = cp.compare_flat(got, _truth(fix), GROUPS)
    q = {f'p{int(x * 100)}': ratios[min(len(ratios) - 1, int(x * len(ratios)))] for x in (0.5, 0.9, 0.99, 1.0)}
    cp.record(f'{tag}_f32', dict(worst=worst, ratio_to_bound_quantiles=q, stats=ws, pl_mean=pl, flat=flat,
                                 reference_flat=ref_flat))
    cp.judge_f32(got, fix, factor=F32_FACTOR, group_factor=F32_GROUP_FACTOR)
    cp.judge_stats_f32(stats, fix)
    cp.judge_pl_mean(got, fix)
    cp.judge_flat({g: v for g, v in flat.items() if g.startswith('grad/')}, ref_flat, floor=1e-4)
    # Parameters after the step: Adam's first step with beta1 = 0 moves an entry by ~lr * sign(g), so an entry
    # whose gradient is within f32 (atomic-order) noise of zero can land 2 * lr from the float64 answer.  The
    # norms stay at 1e-5; the sampled entries get 1e-4 (measured 1.3e-5 at C2, 2.8e-5 at C4 on r02_v4).
    cp.judge_flat({g: v for g, v in flat.items() if not g.startswith('grad/')}, ref_flat, floor=(1e-5, 1e-4))


@pytest.mark.timeout(240)
@pytest.mark.parametrize('tag,dt', [('c1', 'fp16'), ('c1', 'bf16'), ('c2', 'fp16'), ('c4', 'fp16'), ('c5', 'bf16')])
def test_16bit_iteration_vs_reference(tag, dt):
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}.npz'))
    got, _ = cp.run_product(cfg, inp, tape, DEV, fp16_dtype=torch.float16 if dt == 'fp16' else torch.bfloat16)
    cp.save_summary(f'{tag}_{dt}', got)
    res = cp.compare_flat(got, _truth(fix), GROUPS)
    ref = cp.compare_flat(fix, _truth(fix), GROUPS)
    cp.record(f'{tag}_{dt}', dict(flat=res, reference_f32_flat=ref))
    _check_flat(res, ref, FLOOR16[dt])


# ADA at p = 0 (tests/golden/make_golden.py P0_CONFIGS): no discrete augmentation choice can differ between
# f32 and float64, and each fixture carries the float64 conditioning summaries (f64p/: the state nudged by
# half an f32 ulp).  Every tensor is held to max(1e-4, 4 x max(reference f32 error, conditioning, the product's
# own run-to-run spread)) -- its own conditioning, no phase-wide term -- and every tensor the reference's f32
# gets within 1e-4 of float64 must also match the reference's f32 result itself to 3e-4 (or 4x that spread).
P0_TAGS = ['c2p0', 'c4p0', 'c5p0']
# 16-bit at p = 0 (num_fp16_res = 4): floors are 1.5x the worst measured over the three fixtures (round 3,
# profiles/r03_config_parity.jsonl `*_cond` records: fp16 Gmain 0.016 / Greg 0.062 / Dmain 0.13 / Dreg 0.28, bf16
# 0.094 / 0.24 / 0.22 / 0.63).  The 16-bit rounding, not f32 conditioning, sets these: the reference has no
# 16-bit CPU run to compare with, and R1's double backward in bf16 (8-bit mantissa) keeps little of Dreg.
# fp16 'param': 1.5 x the 1.01e-3 that c4p0 D1 measured in r03_v8 (the Dmain bias branch).
P0_FLOOR16 = {
    'fp16': {'grad/Gmain': 0.025, 'grad/Greg': 0.095, 'grad/Dmain': 0.2, 'grad/Dreg': 0.42, 'param': 1.5e-3},
    'bf16': {'grad/Gmain': 0.15, 'grad/Greg': 0.36, 'grad/Dmain': 0.33, 'grad/Dreg': 0.95, 'param': 2e-3},
}


def _cond_flat(fix):
    truth = _truth(fix)
    cond = {k[5:]: v for k, v in fix.items() if k.startswith('f64p/')}
    ref = cp.compare_flat(fix, truth, GROUPS)
    con = cp.compare_flat(cond, truth, GROUPS)
    return {g: (max(ref[g][0], con[g][0]), max(ref[g][1], con[g][1])) for g in GROUPS}, ref, con


# The C4 / C5 fixtures hold batch 2 (C2: 4), so D's minibatch-std groups are pairs, and the random-init D at
# 512^2 / 1024^2 reaches its conv_clamp: its f32 gradients have branch points (sqrt(var + 1e-8) of a pair, the
# clamp mask) that different f32 evaluations take differently.  Measured over 11 runs in 4 processes at C4
# (profiles/r03_c4p0_spread.txt): Dmain's b4.conv.bias is 0.15 off the float64 answer in 9 runs and 2e-4 in 2,
# the same code either way; at C5 the same flips move Dmain's flat vector to 0.09 (reference 0.013).  There the
# D phases are held through their flat vectors (floor 0.15) and the G phases per tensor.
BRANCHY_D = {'c4p0', 'c5p0'}


@pytest.mark.timeout(240)
@pytest.mark.parametrize('tag', P0_TAGS)
def test_f32_iteration_conditioned(tag):
    """f32 iteration at config width with the ADA pipe at p = 0 against the float64 oracle, every tensor held to
    4x the largest of three rounding-sized spreads of the same computation: the reference's own f32 error, the
    float64 answer's shift under a half-ulp nudge of the inputs (f64p), and the product's run-to-run difference
    over two more runs (its atomic reductions change order between runs).  Tensors the reference gets right to 1e-4 must also
    match the reference's f32 result directly."""
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}.npz'))
    got, stats = cp.run_product(cfg, inp, tape, DEV, aug_p=cfg['aug_p'])
    reruns, rerun_stats = [], []
    for _ in range(2):        # two more runs: the product's own run-to-run spread, per tensor
        cfg2, inp2, tape2, _ = cp.load_fixture(load(f'train_{tag}.npz'))
        g2, st2 = cp.run_product(cfg2, inp2, tape2, DEV, aug_p=cfg2['aug_p'])
        reruns.append(g2)
        rerun_stats.append(st2)
    got2 = reruns
    cp.save_summary(f'{tag}_f32', got)
    worst, rows = cp.judge_cond(got, fix, check=False, rerun=got2)
    nref, wref, kref = cp.judge_vs_reference(got, fix, check=False, rerun=got2)
    spread, ref_flat, cond_flat = _cond_flat(fix)
    flat = cp.compare_flat(got, _truth(fix), GROUPS)
    rr_flat = [cp.compare_flat(r, got, GROUPS) for r in reruns]
    rerun_flat = {g: (max(r[g][0] for r in rr_flat), max(r[g][1] for r in rr_flat)) for g in GROUPS}
    spread = {g: (max(spread[g][0], rerun_flat[g][0]), max(spread[g][1], rerun_flat[g][1])) for g in GROUPS}
    cp.record(f'{tag}_f32_cond', dict(worst=worst, top=rows[:8], max_bound={g: w[2] for g, w in worst.items()},
                                      vs_reference=(nref, wref, kref), flat=flat, reference_flat=ref_flat,
                                      conditioning_flat=cond_flat, rerun_flat=rerun_flat))
    if tag in BRANCHY_D:
        # G phases per tensor; D phases through their flat vectors only (see BRANCHY_D)
        # G's gradients flow back through D, so they inherit D's branch flips: up to 5 % of the G tensors may
        # leave their own bound (c5p0, r03_v1: 13 of 543, worst 3.1x, b8.conv0.noise_strength at the 1e-4 floor)
        cp.judge_cond(got, fix, rerun=got2, groups=('grad/Gmain', 'grad/Greg', 'G1/', 'Gema1/'), max_out=0.05)
        # the direct check against the reference's f32 at 3e-3 here, not 3e-4: when both product runs land in one
        # branch of D and the reference in the other, every G gradient moves together (r03_v8 c5p0: 32 of 114 Gmain
        # tensors out of the 3e-4 bound, the first at 7.3e-4; the same tree passed on the next run, r03_v9) and
        # the rerun spread cannot widen the bound; a wrong layer is off by O(1)
        cp.judge_vs_reference(got, fix, rerun=got2, groups=('grad/Gmain', 'grad/Greg'), tol=3e-3)
        cp.judge_flat({g: v for g, v in flat.items() if g in ('grad/Dmain', 'grad/Dreg')}, spread, floor=0.15)
        cp.judge_flat({g: v for g, v in flat.items() if g in ('D1',)}, spread, floor=(1e-5, 2e-3))
        flat = {g: v for g, v in flat.items() if g not in ('grad/Dmain', 'grad/Dreg', 'D1')}
    else:
        cp.judge_cond(got, fix, rerun=got2)
        cp.judge_vs_reference(got, fix, rerun=got2)
        cp.judge_stats_f32(stats, fix, rerun_stats=rerun_stats)
    cp.judge_pl_mean(got, fix)
    cp.judge_flat({g: v for g, v in flat.items() if g.startswith('grad/')}, spread, floor=1e-4,
                  factor=5.0 if tag in BRANCHY_D else 3.0)
    cp.judge_flat({g: v for g, v in flat.items() if not g.startswith('grad/')}, spread, floor=(1e-5, 1e-4))


@pytest.mark.timeout(240)
@pytest.mark.parametrize('tag,dt', [('c2p0', 'fp16'), ('c4p0', 'fp16'), ('c5p0', 'bf16'), ('c2p0', 'bf16')])
def test_16bit_iteration_conditioned(tag, dt):
    cfg, inp, tape, fix = cp.load_fixture(load(f'train_{tag}.npz'))
    got, _ = cp.run_product(cfg, inp, tape, DEV, fp16_dtype=torch.float16 if dt == 'fp16' else torch.bfloat16,
                            aug_p=cfg['aug_p'])
    cp.save_summary(f'{tag}_{dt}', got)
    res = cp.compare_flat(got, _truth(fix), GROUPS)
    spread, ref_flat, cond_flat = _cond_flat(fix)
    cp.record(f'{tag}_{dt}_cond', dict(flat=res, reference_f32_flat=ref_flat, conditioning_flat=cond_flat))
    _check_flat(res, spread, P0_FLOOR16[dt])


class _RecordingTape(cp.Tape):
    """A tape whose replay() records instead: the product draws the sequence itself."""
    def replay(self):
        return self._patched('record')

    @property
    def pos(self):
        return len(self.entries)

    @pos.setter
    def pos(self, v):
        pass


@pytest.mark.timeout(240)
@pytest.mark.parametrize('tag,batch,dt', [('c4', 16, torch.float16), ('c5', 8, torch.bfloat16)])
def test_full_batch_run(tag, batch, dt):
    """The configuration's full per-GPU batch (no CPU evaluation fits here): every reported statistic and
    every gradient / parameter norm finite, and every phase produced non-zero gradients."""
    cfg, _, _, _ = cp.load_fixture(load(f'train_{tag}.npz'))
    cfg = dict(cfg, batch=batch)
    got, stats = cp.run_product(cfg, cp.make_inputs(cfg), _RecordingTape(seed=23), DEV, fp16_dtype=dt)
    for n, v in stats:
        assert np.isfinite(v).all(), f'{n} not finite'
    for k, v in got.items():
        if k.endswith('/norm'):
            assert np.isfinite(v), k
    for ph in cp.PHASES:
        assert any(k.startswith(f'grad/{ph}/') and got[k] > 0 for k in got if k.endswith('/norm')), ph
