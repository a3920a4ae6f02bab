"""Do captured random draws replay the eager draws?  Two graphs (A: the draw kinds of Gmain -- noise randn,
style-mixing rand / random_, ADA rand / randint / normal_ on float32 and float16 -- and B: a second set) are
captured once, then per iteration `manual_seed(s); replay A; replay B` is compared with `manual_seed(s); eager A;
eager B`, element for element.  Usage: python tools/rng_graph_check.py"""
import torch

dev = torch.device('cuda', 0)


def draws_a(out):
    out[0].copy_(torch.randn([32, 1, 64, 64], device=dev))
    out[1].copy_(torch.rand([], device=dev))
    out[2].copy_(torch.empty([], dtype=torch.int64, device=dev).random_(1, 14))
    out[3].copy_(torch.rand([32, 1, 1, 1], device=dev))
    out[4].copy_(torch.randint(0, 4, [32], device=dev))
    out[5].copy_(torch.randn_like(out[5]))
    out[6].normal_()
    out[7].copy_(torch.randn_like(out[7]) / 32.0)


def draws_b(out):
    out[0].copy_(torch.randn([16, 512], device=dev))
    out[1].copy_(torch.rand([32, 3], device=dev) * 2 - 1)


def bufs_a():
    return [torch.zeros([32, 1, 64, 64], device=dev), torch.zeros([], device=dev),
            torch.zeros([], dtype=torch.int64, device=dev), torch.zeros([32, 1, 1, 1], device=dev),
            torch.zeros([32], dtype=torch.int64, device=dev), torch.zeros([32, 1, 128, 128], dtype=torch.float16, device=dev),
            torch.zeros([1000], device=dev),
            torch.zeros([16, 1, 32, 32], device=dev).contiguous(memory_format=torch.channels_last)]


def bufs_b():
    return [torch.zeros([16, 512], device=dev), torch.zeros([32, 3], device=dev)]


ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
sa, sb = bufs_a(), bufs_b()
torch.manual_seed(0)
draws_a(sa)
draws_b(sb)          # eager warm-up
torch.cuda.synchronize()
with torch.cuda.graph(ga):
    draws_a(sa)
with torch.cuda.graph(gb):
    draws_b(sb)
bad = 0
for it in range(4):
    torch.manual_seed(100 + it)
    ga.replay()
    gb.replay()
    got = [t.clone() for t in sa + sb]
    ea, eb = bufs_a(), bufs_b()
    torch.manual_seed(100 + it)
    draws_a(ea)
    draws_b(eb)
    diffs = [float((a.double() - b.double()).abs().max()) for a, b in zip(got, ea + eb)]
    bad += sum(d != 0 for d in diffs)
    print(f'iteration {it}: max |replay - eager| per draw {diffs}', flush=True)
print('RNG replay == eager' if bad == 0 else f'RNG replay differs from eager in {bad} draws', flush=True)
