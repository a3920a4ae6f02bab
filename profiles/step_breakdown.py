"""Per-step kernel time by category from a rocprofv3 kernel trace of bench.py (the timed graph-replay
steps just before the roofline launches).  Usage: python profiles/step_breakdown.py <trace.csv> <ms_per_step>"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
ms = float(sys.argv[2])
# the roofline measures 23 launches of the 256^2 layer (the ring C=64 kernel since r03, the persistent one in
# r02, the halo kernel before) then 23 of the 32^2 layer (halo kernel) at the end of the run
c64 = [r for r in rows if 'conv3x3_c64r' in r['Kernel_Name']] or [r for r in rows if 'conv3x3_c64p' in r['Kernel_Name']]
halo = [r for r in rows if 'conv3x3_halo' in r['Kernel_Name']]
if len(c64) > 23:
    t_end = int(c64[-23]['Start_Timestamp'])
else:
    t_end = int(halo[-23 - 23]['Start_Timestamp']) if len(halo) > 46 else int(halo[0]['Start_Timestamp'])
t0 = t_end - int(16 * ms * 1e6)
win = [r for r in rows if t0 <= int(r['Start_Timestamp']) < t_end]


def cat(n):
    for key, name in [('conv3x3_s2g', 'stride-2 GEMM 16-bit (D down)'), ('conv3x3_c32r', 'ring conv 16-bit C=32'),
                      ('conv3x3_up2', 'up-2 conv 16-bit'), ('conv3x3_c64p', 'halo conv 16-bit C=64 persistent'), ('conv3x3_c64r', 'ring conv 16-bit C=64'), ('conv3x3_halo', 'halo conv 16-bit'), ('wgrad3x3', 'halo wgrad 16-bit'),
                      ('conv_fwd_kernel<float', 'generic conv f32'), ('conv_fwd_kernel', 'generic conv 16-bit'),
                      ('conv_wgrad_kernel<float', 'generic wgrad f32'), ('conv_wgrad_kernel', 'generic wgrad 16-bit'),
                      ('layer_bwd', 'layer_bwd'), ('bias_act', 'bias_act'), ('demod', 'demod'), ('Cijk', 'GEMM'),
                      ('conv_finalize', 'conv finalize'), ('rocclr', 'memset/copy'), ('zero_fill', 'memset/copy'), ('multi_tensor', 'optimizer'),
                      ('adam_multi', 'optimizer'), ('lerp_multi', 'optimizer'),
                      ('pack_weight', 'weight pack'), ('infnorm', 'fp16 pre-normalisation'),
                      ('conv1x1_small', '1x1 conv toRGB / fromRGB'), ('wgrad1x1_small', '1x1 conv toRGB / fromRGB'),
                      ('vjp_axpy', 'fused VJP pass'), ('split3', 'f32 operand split'), ('moments', 'statistics'),
                      ('grouped', 'GEMM')]:
        if key in n:
            return name
    if 'upfirdn' in n:
        return 'upfirdn ' + ('f32' if 'float' in n else '16-bit')
    if 'grid_sample' in n or 'reflect' in n or 'zero_region' in n:
        return 'ADA grid sample / pad'
    return 'torch elementwise / reduce / copy' if 'at::native' in n else 'other'


agg = defaultdict(lambda: [0, 0])
for r in win:
    a = agg[cat(r['Kernel_Name'])]
    a[0] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    a[1] += 1
tot = sum(v[0] for v in agg.values())
print(f'{len(win) / 16:.0f} launches / step, {tot / 16e6:.1f} ms kernel time / step (step {ms} ms)')
for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f'{t / 16e6:7.2f} ms/step {n / 16:7.1f} launches/step  {k}')
# the glue families by kernel (what "torch elementwise" and "other" are made of)
glue = defaultdict(lambda: [0, 0])
for r in win:
    if cat(r['Kernel_Name']) in ('torch elementwise / reduce / copy', 'other'):
        g = glue[r['Kernel_Name'][:110]]
        g[0] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        g[1] += 1
print('glue kernels (torch elementwise / other), top 25:')
for k, (t, n) in sorted(glue.items(), key=lambda kv: -kv[1][0])[:25]:
    print(f'{t / 16e6:7.3f} ms/step {n / 16:7.1f} launches/step  {k}')
