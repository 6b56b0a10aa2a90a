#!/bin/bash
# round 6: the top-down share beside the H pair with the dataflow passes, and
# the region's launches alone
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/slant_solo.py 1080 1920 256 2 > gpurun_out/r06_df2_solo_hd.txt 2>&1 || { tail -20 gpurun_out/r06_df2_solo_hd.txt; exit 1; }
cat gpurun_out/r06_df2_solo_hd.txt
timeout -k 10 300 python tools/slant_solo.py 2160 3840 256 2 > gpurun_out/r06_df2_solo_4k.txt 2>&1 || { tail -20 gpurun_out/r06_df2_solo_4k.txt; exit 1; }
cat gpurun_out/r06_df2_solo_4k.txt
bash tools/slant_share.sh hd256 2 "3 4 5 6 7 8" || exit 1
bash tools/slant_share.sh 4k256 1 "3 4 5 6 7" || exit 1
