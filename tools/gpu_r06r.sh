#!/bin/bash
# round 6, call r: FIR strip tile height A/B (SG2_FIR_TH 8 / 12 / 16) -- parity, micro timing, bench; phase timing
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for th in 12 16; do
  SG2_FIR_TH=$th timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py \
      -k "upfirdn or fir" > $O/tests_$th.log 2>&1 || { echo TFAIL $th; tail -30 $O/tests_$th.log; exit 1; }
  tail -1 $O/tests_$th.log
done
for th in 8 12 16; do SG2_FIR_TH=$th timeout -k 10 120 python -u tools/fir_micro.py 2>&1 | grep -v amdgpu.ids | sed "s/^/th=$th /" | tee -a $O/fir.txt | head -4; done
for th in 8 12 8 12 8 16; do
  SG2_FIR_TH=$th timeout -k 10 300 python -u bench.py --steps 48 --no-cpu-baseline --no-roofline > $O/b.log 2>&1 || { echo BFAIL; tail -20 $O/b.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]); print('th', '$th', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
done
timeout -k 10 300 python -u bench.py --steps 32 --no-cpu-baseline --no-roofline --phase-timing > $O/phase.log 2>&1 && tail -1 $O/phase.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['last_phase_ms'])"
