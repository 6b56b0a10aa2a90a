#!/bin/bash
# round 6: the dataflow slanted passes -- slant parity tests, paired A/B
# against the round-5 library (build/base), hop timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py -k slant tests/test_gpu_slant_guard.py tests/test_gpu_schedules.py -m gpu > gpurun_out/r06_df1_tests.log 2>&1 || { tail -40 gpurun_out/r06_df1_tests.log; exit 1; }
tail -3 gpurun_out/r06_df1_tests.log
$T 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_fullsize.py -k "1080 or 4k256_lr or schedules_agree" -m gpu > gpurun_out/r06_df1_full.log 2>&1 || { tail -40 gpurun_out/r06_df1_full.log; exit 1; }
tail -3 gpurun_out/r06_df1_full.log
bash tools/ab.sh hd256 2 build/base/libsgm_hip.so stereo_matching_amd/libsgm_hip.so || exit 1
bash tools/ab.sh 4k256 1 build/base/libsgm_hip.so stereo_matching_amd/libsgm_hip.so || exit 1
SGM_HIP_LIB=build/hops/libsgm_hip.so $T 300 python tools/slant_hops.py > gpurun_out/r06_df1_hops.txt 2>&1 || { tail -20 gpurun_out/r06_df1_hops.txt; exit 1; }
cat gpurun_out/r06_df1_hops.txt
