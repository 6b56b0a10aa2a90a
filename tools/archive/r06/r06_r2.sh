#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py -k slant tests/test_gpu_slant_guard.py -m gpu > gpurun_out/r06_r2_tests.log 2>&1 || { tail -30 gpurun_out/r06_r2_tests.log; exit 1; }
tail -1 gpurun_out/r06_r2_tests.log
bash tools/ab.sh hd256 3 build/prev/libsgm_hip.so stereo_matching_amd/libsgm_hip.so || exit 1
bash tools/ab.sh 4k256 2 build/prev/libsgm_hip.so stereo_matching_amd/libsgm_hip.so || exit 1
