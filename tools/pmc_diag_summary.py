"""Per-kernel summary of the SQ counter pass of tools/gpu_round.sh (step `diag`).

Counters are summed over a dispatch (rocprofv3 reports them per SE / XCD instance), then averaged over the
dispatches of each (kernel, grid).  Derived, per dispatch:
  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 32)   -- MFMA-busy SIMD cycles over all SIMD
              cycles (SQ_BUSY_CYCLES counts per SE: 32 SEs of 8 CUs x 4 SIMDs on MI355X, so x 32 SIMDs/SE);
              on the equal-FLOP shapes of tools/conv_micro.py SQ_VALU_MFMA_BUSY_CYCLES is the same for every
              kernel (151e6 = FLOPs / 1024 per SIMD-cycle), a check of this reading
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE       -- share of LDS cycles lost to conflicts
  wait_any / wait_inst / active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
Usage: python tools/pmc_diag_summary.py <run_counter_collection.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = (r['Kernel_Name'], int(r['Grid_Size']))
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    disp[k].add(r['Dispatch_Id'])
print(f'{"kernel":78s} {"grid":>8s} {"n":>3s} {"mfma_util":>9s} {"lds_confl":>9s} {"wait_any":>8s} {"wait_inst":>9s} {"active":>6s}')
for (name, grid), v in sorted(agg.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
    nd = len(disp[(name, grid)])
    v = {c: x / nd for c, x in v.items()}
    wc = v.get('SQ_WAVE_CYCLES', 0) or 1
    print(f'{name[:78]:78s} {grid:8d} {nd:3d} {v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1, v.get("SQ_BUSY_CYCLES", 1) * 32):9.3f} '
          f'{v.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, v.get("SQ_LDS_IDX_ACTIVE", 1)):9.3f} {v.get("SQ_WAIT_ANY", 0) / wc:8.3f} '
          f'{v.get("SQ_WAIT_INST_ANY", 0) / wc:9.3f} {v.get("SQ_ACTIVE_INST_ANY", 0) / wc:6.3f}')
