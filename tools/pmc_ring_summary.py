"""Per-kernel average of the SQ counter passes of tools/pmc_ring.sh, with derived shares:
  mfma_util  = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 32)   (tools/pmc_diag_summary.py)
  wait_* / active_* = quad-cycle counters over SQ_WAVE_CYCLES
Usage: python tools/pmc_ring_summary.py <dir>"""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f'{sys.argv[1]}/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = (r['Kernel_Name'][:90], int(r['Grid_Size']))
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[(k, r['Counter_Name'])].add(r['Dispatch_Id'])
for k, v in agg.items():
    v = {c: x / max(1, len(disp[(k, c)])) for c, x in v.items()}
    wc = v.get('SQ_WAVE_CYCLES', 1) or 1
    print(f'{k[0]} grid {k[1]}')
    print(f'  mfma_util {v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1, v.get("SQ_BUSY_CYCLES", 1) * 32):.3f}  '
          f'coexec/mfma {v.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / max(1, v.get("SQ_VALU_MFMA_BUSY_CYCLES", 1)):.3f}  '
          f'lds_confl {v.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, v.get("SQ_LDS_IDX_ACTIVE", 1)):.3f}')
    for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_WAIT_INST_LDS', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU',
              'SQ_ACTIVE_INST_LDS', 'SQ_ACTIVE_INST_SCA', 'SQ_ACTIVE_INST_VMEM'):
        print(f'  {c:28s} {v.get(c, 0) / wc:.3f} of wave cycles')
    for c in ('SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_INSTS_MFMA', 'SQ_INST_CYCLES_SALU', 'SQ_LDS_DATA_FIFO_FULL',
              'SQ_LDS_CMD_FIFO_FULL', 'SQ_VMEM_TA_ADDR_FIFO_FULL', 'SQ_VMEM_TA_CMD_FIFO_FULL',
              'SQ_VMEM_WR_TA_DATA_FIFO_FULL', 'SQ_WAVE_CYCLES', 'SQ_BUSY_CYCLES'):
        print(f'  {c:28s} {v.get(c, 0):.4g}')
