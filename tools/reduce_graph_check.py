"""Does torch's multi-block sum replay bit-exactly inside a captured HIP graph?

The toRGB bias gradient of the narrow-output backward (modconv._fast_backward) is dz.sum([0, 2, 3]) over
2M elements into one value: torch splits it over many workgroups (a staging buffer plus a semaphore array that
it zero-fills with a memset issued inside the capture).  test_bench_gpu saw that value differ between two
identical graph-mode runs.  This replays graphs of the same reductions with fresh inputs staged before each
replay and compares every replay against the eager result of the same input.

    python tools/reduce_graph_check.py [replays]
"""
import sys

import torch


def cases(dev):
    return [
        ('torgb_db_256_f16', lambda x: x.sum([0, 2, 3], dtype=torch.float32), (32, 1, 256, 256), torch.float16),
        ('torgb_db_128_f16', lambda x: x.sum([0, 2, 3], dtype=torch.float32), (32, 1, 128, 128), torch.float16),
        ('r1_pen_256_f32', lambda x: x.square().sum([1, 2, 3]), (32, 1, 256, 256), torch.float32),
        ('all_2m_f32', lambda x: x.sum(), (32, 1, 256, 256), torch.float32),
    ]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device('cuda', 0)
    gen = torch.Generator(device=dev).manual_seed(0)
    bad_total = 0
    for name, fn, shape, dt in cases(dev):
        static = torch.randn(shape, device=dev, generator=gen).to(dt).contiguous(memory_format=torch.channels_last)
        for _ in range(3):                       # warm the allocator / kernels outside the capture
            fn(static)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = fn(static)
        bad = stale = 0
        prev = None
        for r in range(reps):
            src = torch.randn(shape, device=dev, generator=gen).to(dt).contiguous(memory_format=torch.channels_last)
            static.copy_(src)
            g.replay()
            ref = fn(src)
            torch.cuda.synchronize()
            if not torch.equal(out, ref):
                bad += 1
                if prev is not None and torch.equal(out, prev):
                    stale += 1
                if bad <= 3:
                    print(f'  {name} replay {r}: graph {out.flatten()[:2].tolist()} eager {ref.flatten()[:2].tolist()}',
                          flush=True)
            prev = ref
        print(f'{name}: {bad} of {reps} replays differ from eager ({stale} equal to the previous input\'s sum)',
              flush=True)
        bad_total += bad
    print('TOTAL_BAD', bad_total)


if __name__ == '__main__':
    main()
