"""HBM traffic per launch of the roofline kernels from two rocprofv3 --pmc passes (tools/gpu_round.sh).

Correction (MI355X_MICROARCH.md, HBM section; cdna_hip_programming.md section 7): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
tools/roofline_only.py launches two shapes: the 256^2 C=64 layer (bench.py's roofline kernel, the
persistent conv3x3_c64p_kernel) and the 32^2 C=512 layer (conv3x3_halo_kernel, the MFMA-bound
reference point).  Launches are grouped by kernel name; the JSON (read by bench.py) carries the
roofline kernel's figure.
Usage: python tools/pmc_traffic.py <gpurun_out/tag> [out.json]"""
import csv
import glob
import json
import sys
from collections import defaultdict

d = sys.argv[1]
ROOFLINE = 'conv3x3_c64p'


def per_kernel(counter):
    files = glob.glob(f'{d}/pmc_{counter}/**/*counter_collection.csv', recursive=True)
    if not files:
        return None
    vals = defaultdict(float)
    name = {}
    for r in csv.DictReader(open(files[0])):
        if r.get('Counter_Name') != counter:
            continue
        key = r.get('Dispatch_Id') or r.get('Correlation_Id')
        vals[key] += float(r['Counter_Value'])
        name[key] = r.get('Kernel_Name', '')
    by = defaultdict(list)
    for k, v in vals.items():
        by[name[k]].append(v)
    return {n: sum(v) / len(v) for n, v in by.items()}, {n: len(v) for n, v in by.items()}


res = {c: per_kernel(c) for c in ('FETCH_SIZE', 'WRITE_SIZE')}
if any(v is None for v in res.values()):
    print('no data')
    sys.exit(0)
out = None
for kname in res['FETCH_SIZE'][0]:
    f = res['FETCH_SIZE'][0][kname]
    w = res['WRITE_SIZE'][0].get(kname, float('nan'))
    hbm = (2 * f + w) * 1024
    print(f'{kname[:90]}\n    {res["FETCH_SIZE"][1][kname]} launches: FETCH {f:.1f} KiB, WRITE {w:.1f} KiB -> '
          f'HBM bytes per launch (2*FETCH + WRITE) = {hbm:.4g} (read {2 * f * 1024:.4g}, write {w * 1024:.4g})')
    if ROOFLINE in kname:
        out = dict(kernel=kname, hbm_bytes_per_launch=round(hbm), fetch_size_kib=f, write_size_kib=w)
if out is not None and len(sys.argv) > 2:
    with open(sys.argv[2], 'w') as fh:
        json.dump(dict(config='sg2_conv3x3 fused 256^2 C=64 N=32 float16', **out,
                       correction='hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts half of '
                                  'wide coalesced reads; MI355X_MICROARCH.md HBM section)'), fh, indent=1)
