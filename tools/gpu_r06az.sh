#!/bin/bash
# round 6, call az: round-6 counter passes on the final tree -- HBM traffic of the roofline launch (FETCH / WRITE),
# the ring kernel's SQ passes
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_round.sh r06az pmc || exit 1
bash tools/pmc_ring.sh gpurun_out/r06az/pmc_ring || exit 1
find gpurun_out/r06az -name '*counter_collection.csv' -size +20M -delete
