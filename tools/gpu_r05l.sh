#!/bin/bash
# round 5, call l: PMC passes on the default ring form (SQ issue mix, HBM bytes) and the conv census by backend
set -o pipefail
O=gpurun_out/r05l
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/pmc_ring.sh $O/pmc_ring > $O/pmc_ring.log 2>&1 || { tail -20 $O/pmc_ring.log; exit 1; }
tail -25 $O/pmc_ring.log
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'conv3x3_(halo|c64p|c64r)' -d "$O/pmc_$c" -o run \
        --output-format csv -- python3 "$R/tools/roofline_only.py" > "$O/pmc_$c.log" 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $O $O/roofline_traffic.json > $O/pmc_traffic.txt 2>&1; cat $O/pmc_traffic.txt
timeout -k 10 400 python -u tools/conv_census.py > $O/conv_census.log 2>&1 || { tail -30 $O/conv_census.log; exit 1; }
head -12 $O/conv_census.log
