#!/bin/bash
# round 5, call p: product at 2^-12-nudged states (C1 / C2, both 16-bit types) for the same-state 16-bit comparison,
# then the SQ counter passes on the stride-2 GEMM
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
export PYTHONUNBUFFERED=1
for tc in "c2 bf16" "c2 fp16" "c1 bf16" "c1 fp16"; do
  timeout -k 10 300 python -u tools/prod_perturbed.py $tc 12 1 2 3 4 5 6 7 8 > $O/pert_$(echo $tc | tr ' ' _).log 2>&1 || { tail -20 $O/pert_$(echo $tc | tr ' ' _).log; exit 1; }
done
ls gpurun_out/pert | wc -l
bash tools/gpu_r05o.sh
