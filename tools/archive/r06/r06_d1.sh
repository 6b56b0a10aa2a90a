#!/bin/bash
# round 6: two chains per wave at D = 64 -- parity, paired timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10"
SGM_HIP_LIB=build/dual/libsgm_hip.so $T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_real_texture.py -k "64 and not 640" -m gpu > gpurun_out/r06_d1_tests.log 2>&1 || { tail -40 gpurun_out/r06_d1_tests.log; exit 1; }
tail -2 gpurun_out/r06_d1_tests.log
bash tools/ab.sh k64 4 stereo_matching_amd/libsgm_hip.so build/dual/libsgm_hip.so || exit 1
