#!/bin/bash
# round 5, call x: SQ counter passes on the 16-bit weight-gradient kernels (stride 1 and stride 2 bench shapes)
set -o pipefail
O=gpurun_out/r05x
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INSTS_MFMA"
for shape in "64 128 128 1" "32 64 128 2"; do
  tag=$(echo $shape | tr ' ' _)
  mkdir -p $O/$tag
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'wgrad3x3' -d "$O/$tag/p$i" -o run --output-format csv \
        -- python3 tools/wgrad_only.py $shape > "$O/$tag/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/$tag/p$i.log"; exit 1; }
  done
  python3 tools/pmc_ring_summary.py "$O/$tag" | tee "$O/$tag/summary.txt"
done
