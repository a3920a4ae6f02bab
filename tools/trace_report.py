"""Per-kernel time of each part of a rocprofv3 kernel trace of tools/trace_parts.py.  With the run's log (its
'PART <name> <monotonic ns> <boottime ns>' lines) each part is the kernels from its mark to the first idle gap
of > 100 ms after it (the traced run; the warm-up runs come before the mark); without it, sections split at
idle gaps.  Usage: python tools/trace_report.py <dir> [top] [--log trace.log] [--calls]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 25
f = sorted(glob.glob(f'{d}/**/*kernel_trace.csv', recursive=True))[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
marks = []
if '--log' in sys.argv:
    for line in open(sys.argv[sys.argv.index('--log') + 1]):
        if line.startswith('PART '):
            p = line.split()
            marks.append((p[1], [int(x) for x in p[2:]]))
sections = []
if marks:
    t0, t1 = int(rows[0]['Start_Timestamp']), int(rows[-1]['End_Timestamp'])
    clk = next((i for i in range(len(marks[0][1])) if t0 <= marks[0][1][i] <= t1), 0)
    for name, ts in marks:
        sec, last = [], None
        for r in rows:
            s = int(r['Start_Timestamp'])
            if s < ts[clk]:
                continue
            if last is not None and s - last > 100e6:
                break
            sec.append(r)
            last = int(r['End_Timestamp'])
        sections.append((name, sec))
else:
    cur, last = [], None
    for r in rows:
        s = int(r['Start_Timestamp'])
        if last is not None and s - last > 100e6:
            sections.append((str(len(sections)), cur))
            cur = []
        cur.append(r)
        last = int(r['End_Timestamp'])
    sections.append((str(len(sections)), cur))


def short(n):
    return n.replace('(anonymous namespace)::', '').replace('sg2::', '')[:100]


for name, sec in sections:
    if not sec:
        print(f'\n=== {name}: no kernels')
        continue
    tot = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in sec)
    span = int(sec[-1]['End_Timestamp']) - int(sec[0]['Start_Timestamp'])
    print(f'\n=== {name}: {len(sec)} kernels, busy {tot / 1e6:.2f} ms, span {span / 1e6:.2f} ms')
    agg = defaultdict(lambda: [0, 0])
    for r in sec:
        k = short(r['Kernel_Name'])
        agg[k][0] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        agg[k][1] += 1
    for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f'  {t / 1e3:9.1f} us {n:5d}x  {100 * t / tot:5.1f}%  {k}')
    if '--calls' in sys.argv:
        for r in sec:
            t = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            if t > 30e3:
                print(f'    {t / 1e3:8.1f} us grid {r.get("Grid_Size_X", "?")},{r.get("Grid_Size_Y", "")},'
                      f'{r.get("Grid_Size_Z", "")} {short(r["Kernel_Name"])}')
