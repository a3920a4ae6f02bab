"""Where the ring C=64 kernel's loop spends its cycles: run the roofline launch (bench._layer_launch, 256^2 C=64 bs32
fused) under a diagnostic build of conv3x3.hip with SG2_RDIAG=512 (s_memtime stamps around each loop phase, summed
per wave, written once at the end) and print the mean cycles per tile of each phase, over all waves.
    bash tools/ring_diag.sh build  (BITS=512)       SG2HIP_LIB=tools/diag_libs/libsg2hip_r512.so python tools/ring_stamps.py
Phases: 0 issue next tile's DMAs (+ tile decode) | 1 MFMAs issued | 2 epilogue + stores issued | 3 DMA wait |
4 barrier.  (s_memtime counts shader clocks; the stamps cost ~10 % themselves.)"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'gan-track_amd'), ROOT]
import bench  # noqa: E402
import sg2hip  # noqa: E402

dev = torch.device('cuda', 0)
for _ in range(3):
    ms, fl, by = bench._layer_launch(dev, 256, 64, torch.float16)
print(f'launch {ms:.4f} ms (diag build, stamps on)', flush=True)
lib = sg2hip.lib()
f = lib.sg2_diag_ring_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
buf = np.zeros(4096 * 10, dtype=np.uint64)
assert f(buf.ctypes.data, buf.nbytes) == 0
r = buf.reshape(4096, 10)
r = r[r[:, 5] > 0]
ntile = (r[:, 7] & 0xffff).astype(np.float64)
names = ['issue DMAs', 'MFMAs', 'epilogue+stores', 'DMA wait', 'barrier']
tot = r[:, 6].astype(np.float64) - r[:, 5].astype(np.float64)
print(f'waves {len(r)}, tiles per wave {ntile.mean():.1f}, cycles per tile {np.mean(tot / ntile):.0f} '
      f'(span of all waves {int(r[:, 6].max() - r[:, 5].min())} cycles)')
for ph in range(5):
    v = r[:, ph].astype(np.float64) / ntile
    print(f'  {ph} {names[ph]:16s} mean {v.mean():7.0f}  p10 {np.percentile(v, 10):7.0f}  p90 {np.percentile(v, 90):7.0f}')
hw = (r[:, 7] >> 32).astype(np.int64)
simd = (hw >> 4) & 3
wave_slot = hw & 15
xcc = ((r[:, 7] >> 16) & 0xffff).astype(np.int64) & 0xf
dt_clk = r[:, 6].astype(np.float64) - r[:, 5].astype(np.float64)
dt_rt = (r[:, 9].astype(np.float64) - r[:, 8].astype(np.float64)) / 100e6          # s_memrealtime: 100 MHz
st_rt = (r[:, 8].astype(np.float64) - r[:, 8].min()) / 100e6 * 1e6
print(f'in-kernel clock {np.median(dt_clk / dt_rt) / 1e9:.3f} GHz (median over waves; p10 '
      f'{np.percentile(dt_clk / dt_rt, 10) / 1e9:.3f}, p90 {np.percentile(dt_clk / dt_rt, 90) / 1e9:.3f}); wave lifetime '
      f'{np.median(dt_rt) * 1e3:.4f} ms median, {dt_rt.max() * 1e3:.4f} max; start spread {st_rt.max():.1f} us')
lt = dt_rt * 1e3
print('wave lifetime ms percentiles p10/p50/p90/p99/max', ' '.join(f'{np.percentile(lt, q):.4f}' for q in (10, 50, 90, 99, 100)))
xc = ((r[:, 7] >> 16) & 0xffff).astype(np.int64) & 0xf
print('per-XCD median / max lifetime ms', ' '.join(f'{np.median(lt[xc == x]):.4f}/{lt[xc == x].max():.4f}' for x in range(8)))
print('per-XCD clock GHz', ' '.join(f'{np.median((dt_clk / dt_rt)[xc == x]) / 1e9:.3f}' for x in range(8)))
print('simd histogram', np.bincount(simd, minlength=4).tolist(), 'xcc histogram', np.bincount(xcc, minlength=8).tolist())
