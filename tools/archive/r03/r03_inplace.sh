#!/bin/bash
# in-place final cost volume: parity (GPU suite's frame tests with the
# in-place variant) + paired A/B (default | in place, nt C_h | in place, cached C_h)
set -o pipefail
mkdir -p gpurun_out
SGM_HIP_LIB=build/ipc/libsgm_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fullsize.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_schedules.py \
  tests/test_gpu_bm.py > gpurun_out/r03_inplace_tests.log 2>&1 || { tail -30 gpurun_out/r03_inplace_tests.log; exit 1; }
tail -2 gpurun_out/r03_inplace_tests.log
for c in k128 k128lr hd256; do
  bash tools/ab.sh $c 3 stereo_matching_amd/libsgm_hip.so build/ipn/libsgm_hip.so build/ipc/libsgm_hip.so || exit 1
done
