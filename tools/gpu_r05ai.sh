#!/bin/bash
# round 5, call ai: counters on the up-2 kernel (edge split) at 32^2 -> 65^2: SQ pass, HBM fetch / write passes
set -o pipefail
O=gpurun_out/r05ai
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INSTS_MFMA"
i=0
for P in "$P1" "$P3" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'conv3x3_up2' -d "$O/p$i" -o run --output-format csv \
      -- python3 tools/up2_only.py > "$O/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/p$i.log"; exit 1; }
done
python3 tools/pmc_ring_summary.py "$O" | tee "$O/summary.txt"
python3 - "$O" <<'PY' | tee -a "$O/summary.txt"
import csv, glob, sys
d = sys.argv[1]
for i, c in ((3, 'FETCH_SIZE'), (4, 'WRITE_SIZE')):
    f = glob.glob(f'{d}/p{i}/**/*counter_collection.csv', recursive=True)[0]
    v = {}
    for r in csv.DictReader(open(f)):
        if r.get('Counter_Name') == c:
            v[r['Dispatch_Id']] = v.get(r['Dispatch_Id'], 0.0) + float(r['Counter_Value'])
    vals = sorted(v.values())
    print(f'{c}: {len(vals)} launches, median {vals[len(vals) // 2]:.0f} KiB per launch')
PY
