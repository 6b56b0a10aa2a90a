#!/bin/bash
# round 6: slanted tile width (compute waves per tile) 13 / 14 / 15, paired
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
SGM_HIP_LIB=build/nw15/libsgm_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py -k slant -m gpu > gpurun_out/r06_nw_tests.log 2>&1 || { tail -30 gpurun_out/r06_nw_tests.log; exit 1; }
tail -1 gpurun_out/r06_nw_tests.log
bash tools/ab.sh hd256 3 stereo_matching_amd/libsgm_hip.so build/nw15/libsgm_hip.so build/nw13/libsgm_hip.so || exit 1
bash tools/ab.sh 4k256 1 stereo_matching_amd/libsgm_hip.so build/nw15/libsgm_hip.so build/nw13/libsgm_hip.so || exit 1
