"""FETCH_SIZE calibration for the persistent C=64 conv's half-line reads (tools/pmc_calib.py, run by
tools/gpu_round.sh calib).  Reads the calib_<lib>_<counter> rocprofv3 outputs and writes the read factor
(true read bytes per FETCH_SIZE byte) that tools/pmc_traffic.py applies to conv3x3_c64p:

  * the whole-line copy (__amd_rocclr_copyBuffer, reads exactly |x|) checks the guide's x2 rule;
  * the read-only build (d3: MFMAs and stores compiled out) reads x in the kernel's own pattern.  It reads
    every byte of x (and the noise and weights) at least once, so |x| + |noise| + |w| over its FETCH_SIZE is
    a LOWER bound on the pattern's factor; 2 (the whole-line rule) is the upper bound, reached only if
    every half-line were a separate 128-byte fetch.
Usage: python tools/pmc_calib_summary.py gpurun_out/<tag> [out.json]"""
import csv
import glob
import json
import sys
from collections import defaultdict

d = sys.argv[1]
X_BYTES = 32 * 64 * 256 * 256 * 2
NOISE_BYTES = 32 * 256 * 256 * 2
W_BYTES = 64 * 64 * 9 * 2


def kib(lib, counter, pat):
    f = glob.glob(f'{d}/calib_{lib}_{counter}/**/*counter_collection.csv', recursive=True)
    vals, name = defaultdict(float), {}
    for r in csv.DictReader(open(f[0])):
        if r['Counter_Name'] == counter:
            vals[r['Dispatch_Id']] += float(r['Counter_Value'])
            name[r['Dispatch_Id']] = r['Kernel_Name']
    v = [x for k, x in vals.items() if pat in name[k]]
    return sum(v) / len(v) * 1024


copy_f = kib('default', 'FETCH_SIZE', 'copyBuffer')
base_f, base_w = kib('default', 'FETCH_SIZE', 'c64p'), kib('default', 'WRITE_SIZE', 'c64p')
d3_f = kib('d3', 'FETCH_SIZE', 'c64p')
lo = (X_BYTES + NOISE_BYTES + W_BYTES) / d3_f
print(f'whole-line copy of |x| = {X_BYTES / 1e6:.1f} MB: FETCH {copy_f / 1e6:.1f} MB -> factor {X_BYTES / copy_f:.3f} '
      f'(the guide\'s x2 rule)')
print(f'read-only c64p build (d3): FETCH {d3_f / 1e6:.1f} MB for >= {(X_BYTES + NOISE_BYTES + W_BYTES) / 1e6:.1f} MB '
      f'read -> half-line factor >= {lo:.3f} (<= 2)')
print(f'full c64p launch: FETCH {base_f / 1e6:.1f} MB, WRITE {base_w / 1e6:.1f} MB')
print(f'  reads = {lo:.3f} x FETCH = {lo * base_f / 1e6:.1f} MB ({lo * base_f / (X_BYTES + NOISE_BYTES):.3f} x x+noise); '
      f'at the x2 rule {2 * base_f / 1e6:.1f} MB')
if len(sys.argv) > 2:
    json.dump(dict(kernel='conv3x3_c64p', fetch_factor=round(lo, 4), fetch_factor_upper=2.0,
                   copy_factor=round(X_BYTES / copy_f, 4), d3_fetch_bytes=round(d3_f), note=__doc__.split('\n\n')[0]),
              open(sys.argv[2], 'w'), indent=1)
