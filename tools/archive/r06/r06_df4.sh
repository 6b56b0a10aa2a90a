#!/bin/bash
# round 6: why the sweep's HD256 frame (10.7 ms) and bench's (12.1 ms) differ
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 300"
NFR=6 $T python tools/slant_sweep.py "4 8" 1080x1920x256x2 || exit 1
NFR=20 $T python tools/slant_sweep.py "4 8" 1080x1920x256x2 || exit 1
bash tools/slant_share.sh hd256 1 "4 8" || exit 1
bash tools/ab.sh hd256 1 stereo_matching_amd/libsgm_hip.so || exit 1
