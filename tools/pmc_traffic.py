"""HBM traffic per launch of the roofline kernel from two rocprofv3 --pmc passes (tools/gpu_round.sh).

Correction (MI355X_MICROARCH.md, HBM section; cdna_hip_programming.md section 7): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
Only the launches of the roofline shape are averaged (the largest grid of the kernel in the run).
Usage: python tools/pmc_traffic.py <gpurun_out/tag> [out.json]
With out.json, writes {"config": <bench.roofline launch key>, "hbm_bytes_per_launch": ...} for bench.py."""
import json
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]


def per_dispatch(counter):
    files = glob.glob(f'{d}/pmc_{counter}/**/*counter_collection.csv', recursive=True)
    if not files:
        return None
    vals = defaultdict(float)
    grid = {}
    for r in csv.DictReader(open(files[0])):
        if r.get('Counter_Name') != counter:
            continue
        key = r.get('Dispatch_Id') or r.get('Correlation_Id')
        vals[key] += float(r['Counter_Value'])
        grid[key] = int(r.get('Grid_Size') or r.get('Grid_Size_X') or 0)
    return vals, grid


out = {}
for c in ('FETCH_SIZE', 'WRITE_SIZE'):
    res = per_dispatch(c)
    if res is None:
        print(f'{c}: no data')
        continue
    vals, grid = res
    gmax = max(grid.values())
    sel = [v for k, v in vals.items() if grid[k] == gmax]
    out[c] = sum(sel) / len(sel)
    print(f'{c}: {len(sel)} launches at grid {gmax}, mean {out[c]:.1f} KiB per launch')
if len(out) == 2:
    hbm = (2 * out['FETCH_SIZE'] + out['WRITE_SIZE']) * 1024
    print(f'HBM bytes per launch (2*FETCH + WRITE) = {hbm:.4g}  (read {2 * out["FETCH_SIZE"] * 1024:.4g}, '
          f'write {out["WRITE_SIZE"] * 1024:.4g})')
    if len(sys.argv) > 2:
        with open(sys.argv[2], 'w') as f:
            json.dump({'config': 'sg2_conv3x3 fused 256^2 C=64 N=32 float16', 'hbm_bytes_per_launch': round(hbm),
                       'fetch_size_kib': out['FETCH_SIZE'], 'write_size_kib': out['WRITE_SIZE'],
                       'correction': 'hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts half of '
                                     'wide coalesced reads; MI355X_MICROARCH.md HBM section)'}, f, indent=1)
