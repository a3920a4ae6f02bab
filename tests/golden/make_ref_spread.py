"""Reference-derived f32 re-evaluations of a phase-isolated fixture (test infrastructure; build container only).

The REFERENCE's own f32 CPU iteration (tests/golden/make_golden.py's harness, same state, inputs and replayed
random draws) evaluated again under conditions that change only its rounding:
  * threads=<k>: torch.set_num_threads(k) -- oneDNN / MKL split their convolution and GEMM reductions by thread
    count, so each count is another f32 summation order of the same reference code;
  * nudge=<e>: every parameter, real image and latent multiplied by (1 +- 2^e) (fixed random signs): the reference
    at a state equal to the fixture's within f32 rounding (e = -24: half an ulp).
Each sample is saved to $GOLD_CACHE/r32_<tag>_<name>.npz (per-tensor summaries as in the fixture);
`merge` folds every sample into train_<tag>_iso.npz as 'r32_<name>/...'.  These are samples of the spread the
reference's own f32 arithmetic has on each tensor: tests/config_parity.py takes them into the f32 bounds in place
of any comparison of the product with itself.

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference/src/models/stylegan3:tests/golden:tests:. \
        python tests/golden/make_ref_spread.py <tag> threads=1 | nudge=-24[:<seed>] | merge
"""
import copy
import glob
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as mg  # noqa: E402  (the reference harness: shims, reference imports)
import torch  # noqa: E402

from golden_init import init_state, summarize, pack, unpack  # noqa: E402
from rngtape import Tape  # noqa: E402

CACHE = os.environ.get('GOLD_CACHE', '/tmp/gold')


def _perturb(t, rel, gen):
    u = torch.randint(0, 2, t.shape, generator=gen).to(t.dtype) * 2 - 1
    return t * (1 + rel * u)


def run(tag, name, threads=None, nudge=None, seed=4242):
    import config_parity as cp
    path = os.path.join(mg.OUT, f'train_{tag}_iso.npz')
    with np.load(path, allow_pickle=False) as f:
        cfg, inp, tape, _ = cp.load_fixture(f)
    if threads:
        torch.set_num_threads(threads)
    torch.manual_seed(0)
    net, augment_mi, loss_mod, training_stats = mg.net, mg.augment_mi, mg.loss_mod, mg.training_stats
    G = net.Generator(z_dim=cfg['z_dim'], c_dim=cfg['c_dim'], w_dim=cfg['w_dim'], img_resolution=cfg['img_resolution'],
                      img_channels=cfg['img_channels'], channel_base=cfg['channel_base'],
                      channel_max=cfg['channel_max'], num_fp16_res=4, conv_clamp=256,
                      fused_modconv_default='inference_only',
                      mapping_kwargs=dict(num_layers=cfg['map_depth'])).train().requires_grad_(False)
    D = net.Discriminator(c_dim=cfg['c_dim'], img_resolution=cfg['img_resolution'], img_channels=cfg['img_channels'],
                          channel_base=cfg['channel_base'], channel_max=cfg['channel_max'], num_fp16_res=4,
                          conv_clamp=256, epilogue_kwargs=dict(mbstd_group_size=cfg['mbstd'])).train().requires_grad_(False)
    init_state(G, seed=1)
    init_state(D, seed=2)
    if nudge is not None:
        gen = torch.Generator().manual_seed(seed)
        with torch.no_grad():
            for m in (G, D):
                for _, p in sorted(m.named_parameters()):
                    p.copy_(_perturb(p, 2.0 ** nudge, gen))
        inp = {k: (_perturb(torch.from_numpy(np.asarray(v, np.float32)), 2.0 ** nudge, gen).numpy()
                   if k in ('real', 'gen_z', 'z') else v) for k, v in inp.items()}
    aug = augment_mi.AugmentPipe(run_dir=None, batch_size=cfg['batch'], **mg.CLARO_AUG).train().requires_grad_(False)
    aug.p.copy_(torch.as_tensor(cfg['aug_p']))
    orig = training_stats.report
    loss_mod.training_stats.report = lambda n_, v: v
    loss = loss_mod.StyleGAN2Loss(device=torch.device('cpu'), G=G, D=D, augment_pipe=aug, r1_gamma=0.4096,
                                  style_mixing_prob=0.9, pl_weight=2, pl_no_weight_grad=True)
    phases = []
    for pname, module, reg in [('G', G, 4), ('D', D, 16)]:
        phases += [dict(name=pname + 'main', module=module, interval=1), dict(name=pname + 'reg', module=module, interval=reg)]
    start = [{k: v.detach().clone() for k, v in m.state_dict().items()} for m in (G, D)]
    out = {}
    T = mg.T
    with tape.replay():
        for pi, ph in enumerate(phases):
            with torch.no_grad():
                for m, sd in zip((G, D), start):
                    for k, v in m.state_dict().items():
                        v.copy_(sd[k])
            for p in ph['module'].parameters():
                p.grad = None
            ph['module'].requires_grad_(True)
            loss.accumulate_gradients(phase=ph['name'], real_img=T(inp['real']), real_c=T(inp['c']),
                                      gen_z=T(inp['gen_z'][pi]), gen_c=T(inp['gen_c'][pi]), gain=ph['interval'],
                                      cur_nimg=1000)
            ph['module'].requires_grad_(False)
            named = [(n_, p) for n_, p in ph['module'].named_parameters() if p.grad is not None]
            flat = torch.cat([p.grad.flatten() for _, p in named])
            torch.nan_to_num(flat, nan=0, posinf=1e5, neginf=-1e5, out=flat)
            out.update(summarize({n_: g.reshape(p.shape) for (n_, p), g in zip(named, flat.split([p.numel() for _, p in named]))},
                                 f'grad/{ph["name"]}'))
            print(tag, name, ph['name'], 'done', flush=True)
    assert tape.pos == len(tape.entries), 'the re-evaluation consumed a different number of random draws'
    loss_mod.training_stats.report = orig
    os.makedirs(CACHE, exist_ok=True)
    np.savez_compressed(os.path.join(CACHE, f'r32_{tag}_{name}.npz'), **pack(out))
    print(tag, name, 'written', flush=True)


def merge(tag):
    path = os.path.join(mg.OUT, f'train_{tag}_iso.npz')
    with np.load(path, allow_pickle=False) as f:
        z = unpack(f)
    # (the oracle-side conditioning terms of round 4 -- a float64 pass at a 2^-20-nudged state 'f64p/' and emulated
    # f32 samples 'e32_<k>/' -- are replaced by these reference re-evaluations and dropped)
    z = {k: v for k, v in z.items() if not k.startswith(('r32_', 'f64p', 'e32_'))}
    names = []
    for fn in sorted(glob.glob(os.path.join(CACHE, f'r32_{tag}_*.npz'))):
        name = os.path.basename(fn)[len(f'r32_{tag}_'):-4]
        with np.load(fn, allow_pickle=False) as f:
            z.update({f'r32_{name}/{k}': v for k, v in unpack(f).items()})
        names.append(name)
    tmp = path + '.tmp.npz'
    np.savez_compressed(tmp, **pack(z))
    os.replace(tmp, path)              # (atomic: a concurrent reader sees the old or the new file)
    print(tag, 'merged', names, flush=True)


if __name__ == '__main__':
    tag, what = sys.argv[1], sys.argv[2]
    if what == 'merge':
        merge(tag)
    elif what.startswith('threads='):
        run(tag, 't' + what.split('=')[1], threads=int(what.split('=')[1]))
    elif what.startswith('nudge='):          # nudge=<log2>[:<seed>]
        spec = what.split('=')[1].split(':')
        e = int(spec[0])
        seed = int(spec[1]) if len(spec) > 1 else 4242
        run(tag, f'n{-e}' + (f's{seed}' if len(spec) > 1 else ''), nudge=e, seed=seed)
