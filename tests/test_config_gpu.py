"""Training parity at every BASELINE.json configuration's real width, on the GPU, against fixtures the REFERENCE
generated (tests/golden/make_golden.py: the reference's fp32 CPU result and the oracle's float64 evaluation of the
same state, inputs and random draws):

  configs[0]    C1  64^2 1-ch bs8, cbase 16384, map 8, c_dim 2 (the Claro yaml)
  configs[1..2] C2  256^2 1-ch, cbase 16384, map 8, c_dim 2, batch 4 of 32
                    (the DP exchange of configs[2]: tests/test_dist_gloo.py)
  configs[3]    C4  512^2 3-ch, cbase 32768, PL + R1, batch 2 of 16
  configs[4]    C5  1024^2 3-ch, cbase 32768, ADA, batch 2 of 8

* train_<tag>_iso.npz, every configuration: each of the four phases (Gmain, Greg, Dmain, Dreg) from the same
  initial state.  f32 per gradient tensor within max(1e-4, 4 x the reference's f32 error on it, 3 x the
  reference's worst in the phase) of float64 (config_parity.judge_f32) and, where the reference's f32 is within
  1e-4, within 3e-4 of the reference's result itself -- the reference's f32 spread measured by re-running the
  reference itself (tests/golden/make_ref_spread.py); the production arithmetic (deterministic reductions) and
  the f32-input MFMA kernels; 16-bit (num_fp16_res = 4, f32 accumulate) per phase, each error measure
  within 2 x the same measure of the reference's own 16-bit error (the oracle's emulation of its fp16 blocks).
* train_<tag>.npz, C1 and C2: one full iteration (phases, lazy-reg Adam, EMA) -- the step semantics.
* full-batch runs of C4 (bs16, fp16) and C5 (bs8, bf16): every statistic / norm finite.

The phase-isolated tests run the product in its production arithmetic, the library's deterministic mode
(sg2hip.deterministic, the training iteration's default: fixed-order reductions, so a result is a function of the code
and the fixture -- tests/test_deterministic_gpu.py checks two runs bitwise equal -- and bitwise the arithmetic bench.py
times).
"""
import re

import numpy as np
import pytest
import torch

from golden_util import load
import config_parity as cp

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)
GROUPS = ['grad/Gmain', 'grad/Greg', 'grad/Dmain', 'grad/Dreg', 'G1', 'D1', 'Gema1']

def _truth(fix):
    return {k[4:]: v for k, v in fix.items() if k.startswith('f64/')}


F32_FACTOR = 4.0
F32_GROUP_FACTOR = 3.0


# The full iteration (every phase after the previous phases' Adam steps) at C1 / C2.  At C4 / C5 widths its later
# phases are chaotic in ANY f32 evaluation: Adam's first step (beta1 = 0) moves every parameter by ~lr * sign(g),
# so each gradient entry whose sign is below f32 resolution moves its parameter by +-lr, and the phases after it
# start from states that differ by that much (the reference's own f32 Dreg bias gradients are up to 4.6x off the
# float64 answer at C4, profiles/r03_c4p0_spread.txt).  There the phase-isolated tests below are the parity
# check; the iteration's step semantics (Adam, EMA, phase order) are held here and by tests/test_train_gpu.py.
@pytest.mark.timeout(240)
@pytest.mark.parametrize('tag', ['c1', 'c2'])
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


# ---------------------------------------------------------------------------------------------- phase-isolated
# tests/golden/train_<tag>_iso.npz: every phase from the same initial state (no optimiser step in between), the
# reference's f32 CPU result and the oracle's float64 answer (make_golden.py `iso:<tag>`).  Each phase's gradients
# are then a function of one fixed state, and the reference's own f32 error collapses to rounding size (C1: Dreg
# flat 1.4e-5 isolated vs 6.9e-4 in the full iteration, r1_penalty 1.1e-4 vs 3.1e-3).  The product runs
# deterministically (sg2hip.deterministic): a bound is met or missed by the code, never by a run's atomic order.
ISO_TAGS = ['c1', 'c2', 'c4', 'c5']
ISO_GROUPS = ['grad/Gmain', 'grad/Greg', 'grad/Dmain', 'grad/Dreg']


def _iso(tag):
    return cp.load_fixture(load(f'train_{tag}_iso.npz'))


# The product is judged in the arithmetic the bench times and in the library's other f32 arithmetic:
#   'det'    the production arithmetic: the split-bf16 products (S3, conv.hip) with the library's fixed-order slot
#            reductions -- the training iteration's default since round 6 (training/trainer.py
#            Trainer(deterministic=True)), so the judged result is bitwise the one bench.py times, and a function of
#            the code and the fixture alone;
#   'exact'  the f32-input MFMA kernels (SG2_F32_EXACT=1), a diagnostic A/B switch that nothing in training or the
#            bench selects.
# 'det' is held to the full bound on every tensor: the bounds come from the reference's own f32 spread (the fixture's
# reference run and its re-evaluations, config_parity._conditioning) and nothing else.  'exact' is held to the
# phase-level checks (flat vector, statistics, pl_mean) and its per-tensor ratios are recorded.
# The float-atomic reductions (Trainer(deterministic=False), an A/B mode since round 6) are not judged here: their
# result moves with the atomics' order: at C4 the Gmain flat measure of four atomic runs spread over 7.6e-5 .. 1.2e-4
# (1.5e-4 on the round-5 driver box) against one deterministic run's 6.1e-5 -- the noise-strength and weight
# gradients are near-cancelling sums over every pixel (tools/atomic_attr.py, profiles/r06a_attr_c4.log).
F32_ARITH = ['det', 'exact']

@pytest.mark.timeout(300)
@pytest.mark.parametrize('arith', F32_ARITH)
@pytest.mark.parametrize('tag', ISO_TAGS)
def test_f32_phases_vs_reference(tag, arith):
    """f32 product (num_fp16_res = 0, the reference's CPU arithmetic), each phase from the fixture's state:
    every gradient tensor within max(1e-4, 4 x the reference's f32 spread on it, 3 x the reference's worst spread
    in the phase) of float64; every tensor the reference gets to 1e-4 within 3e-4 of the reference's f32 result
    itself; each phase's flat vector within max(1e-4, 3 x the reference's); statistics and pl_mean likewise."""
    cfg, inp, tape, fix = _iso(tag)
    got, stats = cp.run_product(cfg, inp, tape, DEV, aug_p=cfg['aug_p'], isolated=True, deterministic=True,
                                f32_exact=arith == 'exact')
    cp.save_summary(f'{tag}_iso_f32_{arith}', got)
    worst, ratios = cp.judge_f32(got, fix, factor=F32_FACTOR, group_factor=F32_GROUP_FACTOR, groups=('grad/',),
                                 check=False)
    ws = cp.judge_stats_f32(stats, fix, check=False)
    nref, wref, kref = cp.judge_vs_reference(got, fix, factor=F32_FACTOR, check=False)
    ref_flat = cp.reference_flat(fix, _truth(fix), ISO_GROUPS)
    flat = cp.compare_flat(got, _truth(fix), ISO_GROUPS)
    q = {f'p{int(x * 100)}': ratios[min(len(ratios) - 1, int(x * len(ratios)))] for x in (0.5, 0.9, 0.99, 1.0)}
    cp.record(f'{tag}_iso_f32_{arith}', dict(worst=worst, ratio_to_bound_quantiles=q, stats=ws, flat=flat,
                                             reference_flat=ref_flat, vs_reference=(nref, wref, kref)))
    cp.judge_stats_f32(stats, fix)
    cp.judge_pl_mean(got, fix)
    cp.judge_flat(flat, ref_flat, floor=1e-4)
    if arith == 'det':       # the production arithmetic, per tensor
        cp.judge_vs_reference(got, fix, factor=F32_FACTOR)
        cp.judge_f32(got, fix, factor=F32_FACTOR, group_factor=F32_GROUP_FACTOR, groups=('grad/',))


# 16-bit (num_fp16_res = 4, the reference's GPU default; f32 accumulation) against the float64 answer of the same
# isolated phases, held to the REFERENCE's own 16-bit error: the fixtures carry the oracle's emulation of the
# reference's fp16 GPU iteration (q16/, qbf/: make_golden.py `emu:<tag>:<dt>`, oracle.sg2_oracle.EMU16 -- every
# tensor and gradient of a use_fp16 block rounded where the reference's is).  The 16-bit error measures are
# heavy-tailed functions of the state (which lrelu masks and 16-bit roundings fall which way), so one draw against
# one draw is no comparison: both sides are evaluated over a set of states and compared as distributions.
#   * Same-state samples (every configuration and type but those listed below: make_golden.py `emu16p`,
#     make_same_state.py): the fixture state and states nudged by (1 +- 2^-12) (seeded signs: 1/16 of a bf16 ulp, so
#     every state redraws the 16-bit rounding pattern), each with its OWN float64 answer (f64p12s<seed>/) and the
#     emulation there (q16p12s<seed>/, qbfp12s<seed>/); the product runs at the same states (config_parity.run_product
#     perturb: the same signs in the same order, rounded to f32).
#   * A fixture without same-state samples for the type falls back to the emulation at half-f32-ulp nudges of the
#     fixture state (q16n<seed>/, qbfn<seed>/: `emu16n`) against the product at one-ulp nudges -- a weaker sample
#     (a half-ulp nudge flips few 16-bit roundings; profiles/r05_nudge16.txt).
# Per phase and error measure -- the relative error of the vector of tensor norms and of the whole flat gradient
# (config_parity.compare_flat), each bounded by the SAME measure only -- the product's median over its states is
# held to EMU_FACTOR x the emulation's median and the product's largest value to EMU_FACTOR x the emulation's largest
# (floor ISO16_FLOOR): the same statistic on both sides (measured r06, the largest product / emulation ratios of
# the maxima 1.42 (C2 bf16 Gmain flat, 0.0695 / 0.0490) and 1.71 (C2 bf16 Dreg norm vector, 0.0410 / 0.0240);
# profiles/r06f_config_parity.jsonl).
# Run in the production arithmetic (deterministic reductions, the bench's).
EMU_FACTOR = 2.0
ISO16_FLOOR = {'fp16': 5e-3, 'bf16': 1e-2}
EMU_KEY = {'fp16': 'q16', 'bf16': 'qbf'}
NUDGES = 4


def _sub(fix, pre):
    return {k[len(pre) + 1:]: v for k, v in fix.items() if k.startswith(pre + '/')}


def _same_states(fix, dt):
    """[(k, seed, truth prefix, emulation prefix)]: the fixture state and every same-state sample in the fixture."""
    out = []
    for p in sorted({k.split('/', 1)[0] for k in fix if re.match(r'f64p\d+s\d+/', k)}):
        m = re.match(r'f64p(\d+)s(\d+)$', p)
        e = f'{EMU_KEY[dt]}p{m.group(1)}s{m.group(2)}'
        if any(k.startswith(e + '/') for k in fix):
            out.append((int(m.group(1)), int(m.group(2)), p, e))
    return [(0, 0, 'f64', EMU_KEY[dt])] + out if out else []


@pytest.mark.timeout(400)
@pytest.mark.parametrize('tag,dt', [('c1', 'fp16'), ('c1', 'bf16'), ('c2', 'fp16'), ('c2', 'bf16'), ('c4', 'fp16'),
                                    ('c5', 'bf16')])
def test_16bit_phases(tag, dt, det=True):
    cfg, inp, tape, fix = _iso(tag)
    assert any(k.startswith(EMU_KEY[dt] + '/') for k in fix), \
        f'train_{tag}_iso.npz has no {EMU_KEY[dt]}/ summaries (make_golden.py emu:{tag}_iso:{dt})'
    states = _same_states(fix, dt)
    fp = torch.float16 if dt == 'fp16' else torch.bfloat16
    runs, refs = [], []
    if states:
        for k, seed, tp, ep in states:
            cfg, inp, tape, _ = _iso(tag)
            got, _ = cp.run_product(cfg, inp, tape, DEV, fp16_dtype=fp, aug_p=cfg['aug_p'], isolated=True,
                                    deterministic=det, perturb=2.0 ** -k if k else 0.0, perturb_seed=seed)
            if not k:
                cp.save_summary(f'{tag}_iso_{dt}_{"det" if det else "atomic"}', got)
            truth = _sub(fix, tp)
            runs.append(cp.compare_flat(got, truth, ISO_GROUPS))
            refs.append(cp.compare_flat(_sub(fix, ep), truth, ISO_GROUPS))
    else:
        truth = _truth(fix)
        for seed in range(NUDGES + 1):
            cfg, inp, tape, _ = _iso(tag)
            got, _ = cp.run_product(cfg, inp, tape, DEV, fp16_dtype=fp, aug_p=cfg['aug_p'], isolated=True,
                                    deterministic=det, perturb=2.0 ** -23 if seed else 0.0, perturb_seed=seed)
            if not seed:
                cp.save_summary(f'{tag}_iso_{dt}_{"det" if det else "atomic"}', got)
            runs.append(cp.compare_flat(got, truth, ISO_GROUPS))
        pres = sorted({k.split('/', 1)[0] for k in fix if k.split('/', 1)[0] == EMU_KEY[dt] or
                       re.match(EMU_KEY[dt] + r'n\d+/', k)})
        refs = [cp.compare_flat(_sub(fix, p), truth, ISO_GROUPS) for p in pres]
    mode = 'det' if det else 'atomic'
    cp.record(f'{tag}_iso_{dt}_{mode}', dict(same_state=bool(states), product=runs, reference_16bit=refs))
    fails = []
    for g in ISO_GROUPS:
        for j, meas in enumerate(('norm-vector', 'flat')):
            pv = [r[g][j] for r in runs]
            ev = [r[g][j] for r in refs]
            for stat, got_v, ref_v in (('median', float(np.median(pv)), float(np.median(ev))),
                                       ('max', float(max(pv)), float(max(ev)))):
                bound = max(ISO16_FLOOR[dt], EMU_FACTOR * ref_v)
                if got_v > bound:
                    fails.append(f'{g} {meas} {stat}: product {got_v:.3g} over {len(pv)} states > {bound:.3g} '
                                 f'(emulated {dt} over {len(ev)} samples: {ref_v:.3g})')
    assert not fails, '; '.join(fails)


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
