#!/bin/bash
# round 6, call ao: multi-rank rehearsal on one GPU (2 ranks on cuda:0, gloo exchange, eager phases)
set -o pipefail
O=gpurun_out/r06ao
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
SG2_BENCH_BACKEND=gloo SG2_BENCH_SHARE_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 16 --warmup 4 --no-cpu-baseline > $O/r2.log 2>&1 || { echo RFAIL; tail -30 $O/r2.log; exit 1; }
grep '^{' $O/r2.log | cut -c1-600
grep '\[bench\]' $O/r2.log | head -5
