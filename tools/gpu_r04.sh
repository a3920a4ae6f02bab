#!/bin/bash
# Round-4 validation session: the new launch-saving paths (fused ADA geometry, grouped affine, one-launch
# statistics, packed ring epilogue) under test, then the glue / conv census and the ring A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04p}
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_deterministic_gpu.py tests/test_config_gpu.py \
    -k "augment or moments or (c64_ring and 45) or c2 or det_iter or iteration" -q --timeout 200 --timeout-method thread \
    > "$O/t.log" 2>&1
rc=$?; tail -3 "$O/t.log"; [ $rc -eq 0 ] || exit $rc
for f in 4 45 4 45; do SG2_C64_RING=$f timeout -k 10 120 python -u tools/ring_ab.py 5 >> "$O/ring_ab.log" 2>&1 || exit 1; done
grep -v amdgpu.ids "$O/ring_ab.log" | grep fused
timeout -k 10 400 python -u tools/glue_census.py > "$O/glue.log" 2>&1 || exit 1
head -3 "$O/glue.log"
timeout -k 10 300 python -u tools/conv_census.py > "$O/conv.log" 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$O/bench.log" 2>&1 || exit 1
tail -1 "$O/bench.log" | cut -c1-200
