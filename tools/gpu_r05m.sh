#!/bin/bash
# round 5, call m: the stride-2 LDS-DMA GEMM (parity, A/B) and the row-mode weight pack
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "s2g or conv3x3_s2 or pack or down_layer" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_trainer_gpu.py -k "pack" > $O/t2.log 2>&1 || { tail -40 $O/t2.log; exit 1; }
tail -2 $O/t2.log
timeout -k 10 300 python -u tools/s2g_ab.py > $O/s2g_ab.log 2>&1 || { tail -20 $O/s2g_ab.log; exit 1; }
cat $O/s2g_ab.log | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "c64_ring and 49" > $O/t3.log 2>&1 || { tail -40 $O/t3.log; exit 1; }
tail -2 $O/t3.log
timeout -k 10 120 python -u tools/ring_ab.py 5 > $O/ring_ab.log 2>&1 || { tail -20 $O/ring_ab.log; exit 1; }
grep -v amdgpu.ids $O/ring_ab.log
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex 'conv3x3_c64r' -d $O/pmc_salu -o run --output-format csv -- python3 tools/roofline_only.py > $O/pmc_salu.log 2>&1 || { tail -5 $O/pmc_salu.log; exit 1; }
echo pmc done
