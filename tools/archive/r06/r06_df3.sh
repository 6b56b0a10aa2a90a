#!/bin/bash
# round 6: slanted (dataflow) vs the default schedules over frame sizes and
# top-down shares (tools/slant_sweep.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python tools/slant_sweep.py "4 6 8" 375x1242x128x1 375x1242x128x2 375x1242x64x2 512x1056x128x2 720x1280x128x2 720x1280x256x2 1080x1920x64x2 1080x1920x128x1 1080x1920x128x2 1080x1920x256x1 1080x1920x256x2 2160x3840x64x2 2160x3840x128x2 2160x3840x256x1 > gpurun_out/r06_df3_sweep.txt 2>&1 || { tail -20 gpurun_out/r06_df3_sweep.txt; exit 1; }
cat gpurun_out/r06_df3_sweep.txt
