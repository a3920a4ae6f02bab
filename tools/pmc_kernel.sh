#!/bin/bash
# Three SQ counter passes (8 SQ counters each, the per-pass limit) over the kernels matching a regex in a command,
# summarised per kernel by tools/pmc_ring_summary.py.
#   gpurun -- 'bash tools/pmc_kernel.sh <out dir> <kernel regex> <python script and args...>'
O=$1; RX=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$O"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INSTS_MFMA"
i=0
for P in "$P1" "$P2" "$P3"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "$RX" -d "$O/p$i" -o run --output-format csv \
        -- python3 "$@" > "$O/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_ring_summary.py" "$O" | tee "$O/summary.txt"
