#!/bin/bash
# HBM-side traffic per kernel from PMC counters (MI355X_MICROARCH.md "HBM"):
# one rocprofv3 pass per counter, kernel trace only, then tools/pmc_reduce.py
# writes per-launch bytes to profiles/pmc_traffic.json.
# Usage (GPU box): GIT_SHA=<commit> bash tools/pmc.sh TAG [config]
set -o pipefail
TAG=${1:-dev}
CFG=${2:-k128}
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_pmc_${C} -o run --output-format csv \
    -- python bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass \
    > gpurun_out/${TAG}_pmc_${C}.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_${C}.log; exit 1; }
done
python tools/pmc_reduce.py "$TAG" "$CFG" && cp profiles/pmc_traffic.json gpurun_out/${TAG}_pmc_traffic.json
