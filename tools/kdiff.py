"""Compare two rocprofv3 kernel_stats.csv files (same workload, two builds or modes): per kernel family (name without
template arguments) total ms and launches in A and B, sorted by B - A.
    python tools/kdiff.py A_kernel_stats.csv B_kernel_stats.csv [top]"""
import csv
import re
import sys


def fam(name):
    n = name.replace('(anonymous namespace)', 'anon')
    m = re.match(r'_ZN3sg212_GLOBAL__N_1(\d+)', n)
    if m:                                   # mangled sg2 kernel: its identifier
        k = int(m.group(1))
        return n[m.end():m.end() + k]
    n = re.sub(r'<.*', '', n)
    n = re.sub(r'\(.*', '', n)
    return n.replace('void ', '').split('::')[-1][:70]


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        f = fam(r['Name'])
        ms, n = out.get(f, (0.0, 0))
        out[f] = (ms + float(r['TotalDurationNs']) / 1e6, n + int(r['Calls']))
    return out


a, b = load(sys.argv[1]), load(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
ta, tb = sum(v[0] for v in a.values()), sum(v[0] for v in b.values())
print(f'total A {ta:.1f} ms, B {tb:.1f} ms, B - A {tb - ta:+.1f} ms')
rows = [(b.get(k, (0, 0))[0] - a.get(k, (0, 0))[0], k) for k in set(a) | set(b)]
for d, k in sorted(rows, key=lambda x: -abs(x[0]))[:top]:
    print(f'{d:+9.2f} ms  A {a.get(k, (0, 0))[0]:8.2f} ms n={a.get(k, (0, 0))[1]:6d}  B {b.get(k, (0, 0))[0]:8.2f} ms '
          f'n={b.get(k, (0, 0))[1]:6d}  {k}')
