#!/bin/bash
# raw map only when asked for + column-major sub maps: parity, then paired A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r03_subcm_tests.log 2>&1 || { tail -40 gpurun_out/r03_subcm_tests.log; exit 1; }
tail -2 gpurun_out/r03_subcm_tests.log
bash tools/ab.sh k128 3 build/prev/libsgm_hip.so stereo_matching_amd/libsgm_hip.so || exit 1
bash tools/ab.sh k128lr 3 build/prev/libsgm_hip.so stereo_matching_amd/libsgm_hip.so || exit 1
bash tools/ab_env.sh k128lr 2 SGM_SUB_CM 1 0 || exit 1
bash tools/ab.sh hd256 2 build/prev/libsgm_hip.so stereo_matching_amd/libsgm_hip.so || exit 1
bash tools/ab.sh 4k256 2 build/prev/libsgm_hip.so stereo_matching_amd/libsgm_hip.so || exit 1
