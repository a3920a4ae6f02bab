"""Which launches the library's zero fills precede (GPU diagnostic, from a rocprofv3 kernel trace of bench.py):
for every zero_fill_kernel dispatch, its grid size (the bytes it clears) and the next two sg2 / torch kernels on the
stream, aggregated per step.    python tools/zero_fill_sites.py <run_kernel_trace.csv> <steps>"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
steps = float(sys.argv[2])
agg = collections.defaultdict(lambda: [0, 0.0])
for i, r in enumerate(rows):
    if 'zero_fill_kernel' not in r['Kernel_Name']:
        continue
    nxt = ' | '.join(rows[j]['Kernel_Name'].replace('sg2::(anonymous namespace)::', '')[:60]
                     for j in range(i + 1, min(i + 3, len(rows))))
    key = (r.get('Grid_Size', r.get('Grid_Size_X', '?')), nxt)
    agg[key][0] += 1
    agg[key][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
tot = sum(v[1] for v in agg.values())
print(f'zero fills: {sum(v[0] for v in agg.values()) / steps:.1f} per step, {tot / steps:.1f} us per step')
for (g, nxt), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f'{t / steps:7.1f} us/step {n / steps:5.2f}/step grid {g:>8}  -> {nxt}')
