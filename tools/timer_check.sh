#!/bin/bash
# the bottom-up pass's time by the library's HIP events
# and by rocprofv3's kernel trace, on the SAME launches, plus untraced runs
# before and after (what the tracer itself costs).  Usage (GPU box):
#   bash tools/timer_check.sh TAG [config]
set -o pipefail
TAG=${1:-dev}; CFG=${2:-4k256}
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --config $CFG --no-cpu-baseline"
timeout -k 10 300 $B > gpurun_out/${TAG}_tc_untraced1.json 2>gpurun_out/${TAG}_tc.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_tc_trace -o run --output-format csv \
  -- $B > gpurun_out/${TAG}_tc_traced.json 2>>gpurun_out/${TAG}_tc.err || exit 1
timeout -k 10 300 $B > gpurun_out/${TAG}_tc_untraced2.json 2>>gpurun_out/${TAG}_tc.err || exit 1
python tools/timer_check.py "$TAG" | tee gpurun_out/${TAG}_timer_check.txt
