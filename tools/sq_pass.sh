#!/bin/bash
# Issue/wait breakdown per kernel from SQ counters (MI355X_MICROARCH.md
# "rocprofv3 PMC slots": WAIT_ANY = parked on s_waitcnt / barrier,
# WAIT_INST_ANY = issue stall, ACTIVE_INST_ANY = issuing; they add up to
# WAVE_CYCLES), plus a GRBM pass for the effective clock.  One rocprofv3 run
# per counter set, kernel trace only; tools/sq_reduce.py prints the table.
# Usage (GPU box): bash tools/sq_pass.sh TAG [config]
set -o pipefail
TAG=${1:-dev}
CFG=${2:-k128}
export TMPDIR=/tmp
mkdir -p gpurun_out
SETS=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
      "GRBM_GUI_ACTIVE GRBM_COUNT")
k=0
for S in "${SETS[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $S --kernel-trace -d gpurun_out/${TAG}_sq_$k -o run --output-format csv \
    -- python bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass \
    > gpurun_out/${TAG}_sq_$k.log 2>&1 || { tail -20 gpurun_out/${TAG}_sq_$k.log; exit 1; }
  k=$((k+1))
done
python tools/sq_reduce.py "$TAG" > gpurun_out/${TAG}_sq_table.txt && cat gpurun_out/${TAG}_sq_table.txt
