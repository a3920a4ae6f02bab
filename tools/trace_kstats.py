"""Per-launch-shape statistics of the kernels matching a pattern in a rocprofv3 kernel_trace.csv.
    python tools/trace_kstats.py run_kernel_trace.csv REGEX [top]
Groups launches by (kernel family, grid size) -> count, total and average duration."""
import csv
import re
import sys

pat = re.compile(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
g = {}
for r in csv.DictReader(open(sys.argv[1])):
    name = r.get('Kernel_Name', '')
    if not pat.search(name):
        continue
    grid = tuple(int(r.get(f'Grid_Size_{a}', 0) or 0) for a in 'XYZ')
    key = (re.sub(r'[<(].*', '', name.replace('void ', '').replace('(anonymous namespace)::', ''))[-40:], grid)
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    c, t = g.get(key, (0, 0.0))
    g[key] = (c + 1, t + d)
tot = sum(t for _, t in g.values())
print(f'{sum(c for c, _ in g.values())} launches, {tot / 1e3:.2f} ms')
for (k, grid), (c, t) in sorted(g.items(), key=lambda x: -x[1][1])[:top]:
    print(f'{t / 1e3:8.2f} ms  n={c:5d}  avg {t / c:8.1f} us  grid {grid}  {k}')
