"""Split a rocprofv3 kernel trace of tools/trace_parts.py into its parts (by idle gaps) and print
per-kernel time of each part.  Usage: python tools/trace_report.py <dir> [top]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
f = sorted(glob.glob(f'{d}/**/*kernel_trace.csv', recursive=True))[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
parts, cur, last = [], [], None
for r in rows:
    s = int(r['Start_Timestamp'])
    if last is not None and s - last > 100e6:   # >100 ms idle = new section
        parts.append(cur)
        cur = []
    cur.append(r)
    last = int(r['End_Timestamp'])
parts.append(cur)
# each part is run 3x (2 warm + 1 traced) with sleeps around the traced run: keep sections after gaps
names = ['synthesis_fwd', 'D_fwd', 'G_fwd_bwd', 'augD_fwd_bwd', 'Gmain', 'Greg', 'Dmain', 'Dreg']
sections = [p for p in parts if p]
print(f'{len(sections)} sections')


def short(n):
    n = n.replace('(anonymous namespace)::', '').replace('sg2::', '')
    return n[:100]


for i, sec in enumerate(sections):
    label = names[i] if len(sections) == len(names) else str(i)
    tot = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in sec)
    span = int(sec[-1]['End_Timestamp']) - int(sec[0]['Start_Timestamp'])
    print(f'\n=== section {i} {label}: {len(sec)} kernels, busy {tot / 1e6:.2f} ms, span {span / 1e6:.2f} ms')
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
                print(f'    {t / 1e3:8.1f} us grid {r.get("Grid_Size_X", r.get("Grid_Size", "?"))},{r.get("Grid_Size_Y", "")},'
                      f'{r.get("Grid_Size_Z", "")} {short(r["Kernel_Name"])}')
