cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/diag
mkdir -p $O
for v in 0 1; do
  SG2_HALO_PERSIST=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex 'conv3x3' -d $O/p$v -o run --output-format csv -- python3 $R/tools/conv_micro.py --which halo --shapes 256x64 --reps 3 > $O/p$v.log 2>&1 || exit 1
  tail -1 $O/p$v.log
done
