"""One trainer per process (GPU): the Claro 32^2 test network for 6 iterations (reg intervals 2) in eager or graph
mode (graphs from iteration 1), parameters saved to gpurun_out/single_<mode>.pt; `compare` prints the largest
difference between the two files.  Separates a graph replay's own result from interference by another trainer's
eager work in the same process (tools/graph_replay_check.py).  Usage: [TAG=_x] python tools/graph_single.py eager|graph, python tools/graph_single.py compare eager_x graph_x;
env OFF=aug,mix,pl,noise (parts switched off), NO_RNG=1 (all four), GRAPH_OPT=0 (Adam stepped after the replay), SG2_BLAS=cublas|cublaslt,
GRAPH_SKIP=Gmain,... (phases kept eager in graph mode)"""
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden'), os.path.join(ROOT, 'gan-track_amd'), ROOT]
OUT = os.path.join(ROOT, 'gpurun_out')
mode = sys.argv[1]
if mode == 'compare':    # compare <tagA> <tagB>: files single_<tag>.pt (tags such as eager, graph_norng)
    a = torch.load(os.path.join(OUT, f'single_{sys.argv[2]}.pt'), weights_only=True)
    b = torch.load(os.path.join(OUT, f'single_{sys.argv[3]}.pt'), weights_only=True)
    diffs = sorted(((float((a[k] - b[k]).abs().max()), k) for k in a), reverse=True)
    num = sum(float((a[k] - b[k]).double().square().sum()) for k in a) ** 0.5
    den = sum(float(a[k].double().square().sum()) for k in a) ** 0.5
    print(f'{sys.argv[3]} vs {sys.argv[2]}, separate processes: rel L2 {num / den:.3g}; worst {diffs[:4]}')
    sys.exit(0)
if os.environ.get('SG2_BLAS'):          # 'cublas' (rocBLAS on ROCm) or 'cublaslt' (hipBLASLt)
    torch.backends.cuda.preferred_blas_library(os.environ['SG2_BLAS'])
from golden_util import load  # noqa: E402
from parity_train import build_product, CLARO_AUG  # noqa: E402
from training import augment_mi, loss as loss_mod, trainer as trainer_mod  # noqa: E402

dev = torch.device('cuda', 0)
z = load('train_claro.npz')
cfg, G, D = build_product(z, dev, False)
G_ema = copy.deepcopy(G).eval()
aug = augment_mi.AugmentPipe(run_dir=None, batch_size=cfg['batch'], **CLARO_AUG).train().requires_grad_(False).to(dev)
# OFF: what to switch off, comma-separated from aug (ADA p = 0), mix (no style mixing), pl (pl_weight 0: no Greg),
# noise (constant synthesis noise); NO_RNG=1 is all four (every random draw then leaves the results unchanged)
OFF = set(filter(None, os.environ.get('OFF', 'aug,mix,pl,noise' if os.environ.get('NO_RNG') == '1' else '').split(',')))
aug.p.copy_(torch.as_tensor(0.0 if 'aug' in OFF else 0.3))
loss = loss_mod.StyleGAN2Loss(device=dev, G=G, D=D, augment_pipe=aug, r1_gamma=0.4096,
                              style_mixing_prob=0.0 if 'mix' in OFF else 0.9, pl_weight=0 if 'pl' in OFF else 2,
                              pl_no_weight_grad=True)
if os.environ.get('PLCONST') == '1':     # the path-length pass's y = randn_like(img) replaced by a fixed pattern
    loss_mod.torch = type('T', (), {k: getattr(torch, k) for k in dir(torch) if not k.startswith('__')})()
    loss_mod.torch.randn_like = lambda t: torch.sin(torch.arange(t.numel(), device=t.device, dtype=t.dtype)).reshape(t.shape)
if 'noise' in OFF:
    _fwd = G.synthesis.forward
    G.synthesis.forward = lambda ws, **kw: _fwd(ws, **{**kw, 'noise_mode': 'const'})
opt = dict(class_name='torch.optim.Adam', lr=0.0025, betas=[0, 0.99], eps=1e-8)
tr = trainer_mod.Trainer(G, D, G_ema, loss, opt, opt, G_reg_interval=2, D_reg_interval=2, batch_size=cfg['batch'],
                         batch_gpu=cfg['batch'], num_gpus=1, rank=0, device=dev, overlap=False, bucket_mb=32)
tr.graph_opt = os.environ.get('GRAPH_OPT', '1') == '1'
_skip = set(filter(None, os.environ.get('GRAPH_SKIP', '').split(',')))   # phases kept eager in graph mode
if _skip:
    _orig = trainer_mod.Trainer._graph_phase

    def _graph_phase(self, phase, ri, rc, gz, gc):
        if phase.name not in _skip:
            return _orig(self, phase, ri, rc, gz, gc)
        phase.opt.zero_grad(set_to_none=True)
        phase.module.requires_grad_(True)
        self._accumulate(phase, ri, rc, gz, gc)
        phase.module.requires_grad_(False)
        return phase.exchange.finish(phase.name, None), False
    trainer_mod.Trainer._graph_phase = _graph_phase
gen = torch.Generator(device=dev)
gen.manual_seed(5)
BENCH = os.environ.get('BENCH_FLOW') == '1'      # bench.py's flow: all four phases captured in one step
for it in range(6):
    if it == 1:
        tr.graphs = mode == 'graph'
        if BENCH:
            tr.batch_idx = 0
    real = torch.rand([cfg['batch'], 1, 32, 32], device=dev, generator=gen) * 2 - 1
    c = torch.nn.functional.one_hot(torch.randint(0, 2, [cfg['batch']], device=dev, generator=gen), 2).float()
    gz = torch.randn([4, cfg['batch'], cfg['z_dim']], device=dev, generator=gen)
    torch.manual_seed(123 + it)
    tr.step([real], [c], [[gz[i]] for i in range(4)], [[c] for _ in range(4)])
torch.cuda.synchronize()
os.makedirs(OUT, exist_ok=True)
torch.save({f'{pre}.{n}': p.detach().cpu() for pre, m in (('G', G), ('D', D), ('G_ema', G_ema))
            for n, p in m.named_parameters()}, os.path.join(OUT, f"single_{mode}{os.environ.get('TAG', '')}.pt"))
if tr.graphs:
    print('captured phases:', sorted(tr._graphs), flush=True)
print(f'{mode}: saved', flush=True)
