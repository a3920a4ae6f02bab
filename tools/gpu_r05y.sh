#!/bin/bash
# round 5, call y: the stride-2 weight gradient's swizzled LDS layout (SG2_WGRAD_SWZ=1) -- parity, timing, conflicts
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
SG2_WGRAD_SWZ=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "wgrad" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for swz in 0 1 0 1; do
  for shape in "32 64 128 2" "64 128 64 2" "64 256 32 2"; do
    tag=swz${swz}_$(echo $shape | tr ' ' _)
    SG2_WGRAD_SWZ=$swz timeout -s KILL 90 rocprofv3 --kernel-trace --stats --kernel-include-regex 'wgrad3x3_s2' -d "$O/$tag" -o run --output-format csv -- python3 tools/wgrad_only.py $shape > $O/$tag.log 2>&1 || { echo "fail $tag"; tail -5 $O/$tag.log; exit 1; }
    f=$(find $O/$tag -name 'run_kernel_stats.csv' | head -1)
    echo "$tag $(python3 -c "import csv,sys; r=[x for x in csv.DictReader(open('$f'))]; print(' '.join(f\"{x['Name'][:40]} avg {float(x['AverageNs'])/1e3:.1f}us n={x['Calls']}\" for x in r))")"
  done
done
for swz in 0 1; do
  SG2_WGRAD_SWZ=$swz timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex 'wgrad3x3_s2' -d "$O/pmc$swz" -o run --output-format csv -- python3 tools/wgrad_only.py 64 128 64 2 > $O/pmc$swz.log 2>&1 || { echo "pmc fail"; tail -5 $O/pmc$swz.log; exit 1; }
done
echo done
