"""Kernel time by family from a rocprofv3 --stats CSV: python tools/fam_sum.py <run_kernel_stats.csv> [per]"""
import csv
import re
import sys
from collections import defaultdict

per = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
fam = defaultdict(lambda: [0.0, 0])
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    m = re.search(r'(conv_fwd_kernel|conv_wgrad_kernel|split3_kernel|conv_finalize_kernel)<?([a-z_0-9]*)', n)
    key = (m.group(1) + '<' + m.group(2) + '>') if m else None
    if 'IDF16' in n or 'DF16' in n:
        key = (m.group(1) if m else n[:40]) + '<f16>'
    if key is None:
        continue
    fam[key][0] += float(r['TotalDurationNs']) / 1e6 / per
    fam[key][1] += int(r['Calls'])
for k, (t, c) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
    print(f'{t:9.3f} ms  n={c:6d}  {k}')
