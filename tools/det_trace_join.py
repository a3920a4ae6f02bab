"""Join det_trace.py's host lines with the det_sum dispatches of a rocprofv3 kernel trace (in order) and print the
time per call shape per step.   python tools/det_trace_join.py calls.txt kernel_trace.csv"""
import collections
import csv
import re
import sys

calls, cyc = [], None
for line in open(sys.argv[1]):
    if line.startswith('CYCLE_BEGIN'):
        cyc = len(calls)
    elif line.startswith('CYCLE_END'):
        end = len(calls)
    m = re.match(r'DETSUM G=(\d+) n=(\d+) S=(\d+) K=(\d+)', line)
    if m:
        calls.append(tuple(int(v) for v in m.groups()))
rows = [r for r in csv.DictReader(open(sys.argv[2])) if 'det_sum_kernel' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
need = sum(2 if k > 1 else 1 for _, _, _, k in calls)
print(f'{len(calls)} calls ({need} launches expected), {len(rows)} det_sum dispatches traced')
assert need == len(rows), 'call / dispatch counts differ'
per = collections.defaultdict(lambda: [0, 0.0])
j = 0
for c_i, (g, n, s, k) in enumerate(calls):
    t = 0.0
    for _ in range(2 if k > 1 else 1):
        r = rows[j]
        t += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        j += 1
    if cyc <= c_i < end:
        per[(g, n, s, k)][0] += 1
        per[(g, n, s, k)][1] += t
tot = sum(v[1] for v in per.values()) / 16
print(f'det_sum per step: {sum(v[0] for v in per.values()) / 16:.1f} calls, {tot / 1e3:.3f} ms')
for (g, n, s, k), (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:40]:
    mb = 4.0 * g * n * (s + 1) / 1e6
    print(f'{t / 16 / 1e3:7.3f} ms/step {c / 16:6.2f}/step avg {t / c:7.1f} us  G={g:5d} n={n:9d} S={s:6d} K={k:4d} '
          f'{mb:8.2f} MB  {mb / (t / c) :6.2f} TB/s')
