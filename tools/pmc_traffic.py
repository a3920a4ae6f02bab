"""HBM traffic per launch of the roofline kernels from two rocprofv3 --pmc passes (tools/gpu_round.sh).

Correction (MI355X_MICROARCH.md, HBM section; cdna_hip_programming.md section 7): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
tools/roofline_only.py launches two shapes: the 256^2 C=64 layer (bench.py's roofline kernel: the ring
conv3x3_c64r_kernel since round 3, the persistent conv3x3_c64p_kernel in round 2) and the 32^2 C=512 layer
(conv3x3_halo_kernel, the MFMA-bound reference point).  Launches are grouped by kernel name; the JSON (read by bench.py) carries the
roofline kernel's figure.
Usage: python tools/pmc_traffic.py <gpurun_out/tag> [out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
ROOFLINE = ('conv3x3_c64r', 'conv3x3_c64p')


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
# The x2 rule is calibrated for whole-line reads (global_load and buffer_load ... lds alike), which is how the ring
# kernel reads (8 whole 128-byte pixel lines per LDS-DMA instruction).  The persistent C=64 conv of round 2 reads
# 64-byte half-lines; its own factor comes from tools/pmc_calib_summary.py (profiles/pmc_calib.json): a lower bound
# measured on its read-only build, the x2 rule the upper bound.
CALIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'profiles', 'pmc_calib.json')
calib = json.load(open(CALIB)) if os.path.exists(CALIB) else None
out = None
for kname in res['FETCH_SIZE'][0]:
    f = res['FETCH_SIZE'][0][kname]
    w = res['WRITE_SIZE'][0].get(kname, float('nan'))
    ff = calib['fetch_factor'] if (calib and calib['kernel'] in kname) else 2.0
    hbm = (ff * f + w) * 1024
    print(f'{kname[:90]}\n    {res["FETCH_SIZE"][1][kname]} launches: FETCH {f:.1f} KiB, WRITE {w:.1f} KiB -> '
          f'HBM bytes per launch ({ff:g}*FETCH + WRITE) = {hbm:.4g} (read {ff * f * 1024:.4g}, write {w * 1024:.4g})'
          + (f'; at the x2 rule {(2 * f + w) * 1024:.4g}' if ff != 2.0 else ''))
    if any(r in kname for r in ROOFLINE) and (out is None or ROOFLINE[0] in kname):
        out = dict(kernel=kname, hbm_bytes_per_launch=round(hbm), hbm_bytes_per_launch_x2_rule=round((2 * f + w) * 1024),
                   fetch_size_kib=f, write_size_kib=w, fetch_factor=ff)
if out is not None and len(sys.argv) > 2:
    with open(sys.argv[2], 'w') as fh:
        json.dump(dict(config='sg2_conv3x3 fused 256^2 C=64 N=32 float16', **out,
                       correction='hbm = (fetch_factor * FETCH_SIZE + WRITE_SIZE) * 1024; ' + (
                           'fetch_factor 2: the guide\'s gfx950 rule for whole-line 16-byte-per-lane reads '
                           '(MI355X_MICROARCH.md HBM section), which is how this kernel reads (LDS-DMA of 8 whole '
                           'pixel lines per instruction)' if out['fetch_factor'] == 2.0 else
                           'fetch_factor from the kernel\'s own read-only calibration (profiles/pmc_calib.json, lower '
                           'bound) -- the guide\'s x2 holds for whole-line reads only')),
                  fh, indent=1)
