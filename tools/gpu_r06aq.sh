#!/bin/bash
# round 6, call aq: BLAS backend A/B for the small FC GEMMs (hipBLASLt default vs rocBLAS)
set -o pipefail
O=gpurun_out/r06aq
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for b in 1 0 1 0; do
TORCH_BLAS_PREFER_HIPBLASLT=$b timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $O/bench_$b.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$b.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_$b.log') if l.startswith('{')][-1]); print('hipblaslt', $b, d['value'], d['ms_per_step'])"
done
TORCH_BLAS_PREFER_HIPBLASLT=0 timeout -k 10 300 python -u tools/glue_time.py 4 > $O/glue_rocblas.txt 2>&1 || { echo GFAIL; tail -20 $O/glue_rocblas.txt; exit 1; }
head -8 $O/glue_rocblas.txt | tail -6
