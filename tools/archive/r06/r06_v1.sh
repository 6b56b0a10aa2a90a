#!/bin/bash
# round 6: the dataflow passes with the re-swept defaults -- GPU tests of the
# changed areas, paired A/B against round 5's library, hop timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_slant_guard.py tests/test_gpu_load_order.py tests/test_cpp_surface.py tests/test_gpu_schedules.py tests/test_gpu_fuzz.py -m gpu > gpurun_out/r06_v1_tests.log 2>&1 || { tail -40 gpurun_out/r06_v1_tests.log; exit 1; }
tail -2 gpurun_out/r06_v1_tests.log
bash tools/ab.sh hd256 3 build/base/libsgm_hip.so stereo_matching_amd/libsgm_hip.so || exit 1
bash tools/ab.sh 4k256 2 build/base/libsgm_hip.so stereo_matching_amd/libsgm_hip.so || exit 1
SGM_HIP_LIB=build/hops/libsgm_hip.so $T 300 python tools/slant_hops.py > gpurun_out/r06_v1_hops.txt 2>&1 || { tail -20 gpurun_out/r06_v1_hops.txt; exit 1; }
cat gpurun_out/r06_v1_hops.txt
