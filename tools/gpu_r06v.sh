#!/bin/bash
# graph memset inventory + bench-step reproducibility test (staged narrow-output sums)
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 300 python -u tools/graph_memsets.py $O/dots > $O/memsets.txt 2>&1 || echo "graph_memsets rc=$?" >> $O/memsets.txt
timeout -k 10 500 python -u -m pytest tests/test_bench_gpu.py -x -v --timeout 450 --timeout-method thread > $O/t.log 2>&1
