#!/bin/bash
# round 5, call r: halo direct epilogue A/B (alternating order) and the bench with / without it
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/halo_direct_ab.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
for d in 0 1 0 1; do
  SG2_HALO_DIRECT=$d timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $O/bench_$d.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$d.log; exit 1; }
  echo "direct=$d $(tail -1 $O/bench_$d.log | cut -c1-160)"
done
