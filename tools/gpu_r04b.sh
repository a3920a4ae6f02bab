#!/bin/bash
# ring A/B, glue / conv census and a bench line (no tests)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04q}
mkdir -p "$O"
cd "$R" || exit 1
for f in 4 45 4 45; do SG2_C64_RING=$f timeout -k 10 120 python -u tools/ring_ab.py 5 >> "$O/ring_ab.log" 2>&1 || exit 1; done
grep -v amdgpu.ids "$O/ring_ab.log" | grep fused
timeout -k 10 400 python -u tools/glue_census.py > "$O/glue.log" 2>&1 || exit 1
head -3 "$O/glue.log"
timeout -k 10 300 python -u tools/conv_census.py > "$O/conv.log" 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$O/bench.log" 2>&1 || exit 1
tail -1 "$O/bench.log" | cut -c1-200
