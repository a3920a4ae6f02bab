#!/bin/bash
# round 5, call z: the pipelined stride-2 weight gradient (parity, A/B, bench)
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "wgrad" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u tools/wgrad_s2p_ab.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
for d in 0 1; do
  SG2_WGRAD_S2P=$d timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $O/bench_$d.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$d.log; exit 1; }
  echo "s2p=$d $(tail -1 $O/bench_$d.log | cut -c1-130)"
done
