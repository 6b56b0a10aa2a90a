#!/bin/bash
# round 6: top-down share and launch order of the concurrent region, slanted sizes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
HFIRST=1 REPS=3 NFR=8 timeout -k 10 1000 python tools/slant_sweep.py "3 4 5 6 8" 1080x1920x256x2 1080x1920x256x1 720x1280x256x2 1080x1920x128x2 2160x3840x128x2 2160x3840x256x1 2160x3840x256x2 > gpurun_out/r06_df6_sweep.txt 2>&1 || { tail -20 gpurun_out/r06_df6_sweep.txt; exit 1; }
cat gpurun_out/r06_df6_sweep.txt
