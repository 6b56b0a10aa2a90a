#!/bin/bash
# load_seg running pointer: parity, then paired timing against the previous build.
set -o pipefail
mkdir -p gpurun_out
SGM_HIP_LIB=build/ls_new/libsgm_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fuzz.py "tests/test_gpu_fullsize.py::test_fullsize_vs_oracle" tests/test_gpu_parity.py \
  > gpurun_out/r03_ls_tests.log 2>&1 || { tail -40 gpurun_out/r03_ls_tests.log; exit 1; }
tail -1 gpurun_out/r03_ls_tests.log
bash tools/ab.sh k128 4 build/ls_base/libsgm_hip.so build/ls_new/libsgm_hip.so || exit 1
bash tools/ab.sh k128lr 2 build/ls_base/libsgm_hip.so build/ls_new/libsgm_hip.so || exit 1
bash tools/ab.sh hd256 1 build/ls_base/libsgm_hip.so build/ls_new/libsgm_hip.so || exit 1
