"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: top kernels and GPU-busy time."""
import csv
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(f'{d}/run_kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows)
calls = sum(int(r['Calls']) for r in rows)
print(f'kernels: {calls} launches, {tot/1e6:.1f} ms GPU time')
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['Percentage']):6.2f}% n={r['Calls']:>6} "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:100]}")
try:
    tr = list(csv.DictReader(open(f'{d}/run_kernel_trace.csv')))
    ts = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in tr)
    busy, cur_s, cur_e = 0, None, None
    for s, e in ts:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = ts[-1][1] - ts[0][0]
    print(f'trace span {span/1e6:.1f} ms, GPU busy {busy/1e6:.1f} ms ({100*busy/span:.1f}%)')
    if len(sys.argv) > 3:   # busy fraction inside the last <tail_ms> of the trace (the timed steps)
        tail = float(sys.argv[3]) * 1e6
        t0 = ts[-1][1] - tail
        busy2, ce = 0, None
        cs = None
        for s_, e_ in ts:
            s_, e_ = max(s_, t0), e_
            if e_ <= t0:
                continue
            if ce is None or s_ > ce:
                if ce is not None:
                    busy2 += ce - cs
                cs, ce = s_, e_
            else:
                ce = max(ce, e_)
        busy2 += ce - cs
        print(f'last {tail/1e6:.0f} ms: GPU busy {busy2/1e6:.1f} ms ({100*busy2/tail:.1f}%)')
except Exception as e:  # noqa: BLE001
    print('no trace:', e)
