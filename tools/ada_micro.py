"""The ADA pipe of the bench configuration alone (GPU diagnostic): 256^2 1-ch, batch 32, p = 0.2, forward +
backward of the geometric stage, 40 iterations; prints the device time per kernel per iteration and, for one
draw, the dynamic extents the 1-D FIR passes compute (lims) next to their static buffers.
    python tools/ada_micro.py [iters] [det]     (det: the deterministic reductions, the training default)"""
import collections
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
from training import augment_mi  # noqa: E402

DEV = torch.device('cuda', 0)


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    if len(sys.argv) > 2 and sys.argv[2] == 'det':
        import sg2hip
        global _DET
        _DET = sg2hip.deterministic(True, device=DEV)            # kept referenced: for the whole run
        _DET.__enter__()
    torch.manual_seed(0)
    aug = augment_mi.AugmentPipe(run_dir=None, batch_size=32, xflip=1, xint=1, scale=1, rotate=1, aniso=1, xfrac=1,
                                 xint_max=0.05, rotate_max=3 / 360, xfrac_std=0.05, scale_std=0.05,
                                 aniso_std=0.05).train().requires_grad_(False).to(DEV)
    aug.p.copy_(torch.as_tensor(0.2))
    x = torch.randn(32, 1, 256, 256, device=DEV, requires_grad=True)
    g = torch.randn(32, 1, 256, 256, device=DEV)
    seen = {}
    orig = torch.empty

    def spy(*a, **k):
        t = orig(*a, **k)
        if k.get('dtype') == torch.int32 and list(a[0] if a and isinstance(a[0], (list, tuple)) else a) == [14]:
            seen['ints'] = t
        return t
    torch.empty = spy
    y = aug(x)
    torch.empty = orig
    torch.cuda.synchronize()
    if 'ints' in seen:
        v = seen['ints'].tolist()
        print(f'margins {v[:4]}  lims (fwd h, fwd v, bwd h, bwd v) {v[4:12]}  dyn_hw {v[12:]}  out {tuple(y.shape)}',
              flush=True)
    for _ in range(5):
        y = aug(x)
        y.backward(g)
    torch.cuda.synchronize()
    if os.environ.get('ADA_NOPROF'):               # under rocprofv3 (counter passes): the iterations only
        for _ in range(iters):
            y = aug(x)
            y.backward(g)
        torch.cuda.synchronize()
        return
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(iters):
            y = aug(x)
            y.backward(g)
        torch.cuda.synchronize()
    per = collections.defaultdict(lambda: [0, 0.0])
    for e in prof.events():
        if e.device_type.name == 'CUDA':
            per[e.name][0] += 1
            per[e.name][1] += e.device_time
    tot = sum(v[1] for v in per.values()) / iters
    print(f'ADA fwd+bwd: {tot:.1f} us of kernels per iteration', flush=True)
    for name, (n, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f'{t / iters:8.1f} us/iter {n / iters:5.1f}/iter avg {t / n:7.1f} us  {name[:110]}', flush=True)


if __name__ == '__main__':
    main()
