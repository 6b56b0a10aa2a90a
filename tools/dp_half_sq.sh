#!/bin/bash
# issue cost per chain step of the two-chains-per-wave DP
# layout (tools/dp_half.hip, chain2: 32 lanes x 4 disparities per chain at
# D = 128) against the production layout (chain1: one chain per wave, 2 per
# lane), from SQ counters, at 375 .. 6144 chains (0.4 .. 6 production waves
# per SIMD).  One rocprofv3 pass per counter set, kernel trace only; the
# table comes from tools/dp_half_sq.py.
# Usage (GPU box; build tools/dp_half first): bash tools/dp_half_sq.sh TAG
set -o pipefail
TAG=${1:-dev}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/dp_half > gpurun_out/${TAG}_dp_half.txt 2>&1 || { cat gpurun_out/${TAG}_dp_half.txt; exit 1; }
SETS=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
      "GRBM_GUI_ACTIVE GRBM_COUNT")
k=0
for S in "${SETS[@]}"; do
  timeout -s KILL 60 rocprofv3 --pmc $S --kernel-trace -d gpurun_out/${TAG}_dpsq_$k -o run --output-format csv \
    -- ./tools/dp_half > gpurun_out/${TAG}_dpsq_$k.log 2>&1 || { tail -20 gpurun_out/${TAG}_dpsq_$k.log; exit 1; }
  k=$((k+1))
done
python tools/dp_half_sq.py "$TAG" > gpurun_out/${TAG}_dp_half_sq.txt && cat gpurun_out/${TAG}_dp_half_sq.txt
