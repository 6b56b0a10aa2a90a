#!/bin/bash
# Final-pass producer buffers (SGM_FINAL_NB 2/3/4): parity of NB=4, then paired timing.
set -o pipefail
mkdir -p gpurun_out
SGM_HIP_LIB=build/nb4/libsgm_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fuzz.py "tests/test_gpu_fullsize.py::test_fullsize_vs_oracle" tests/test_gpu_parity.py \
  > gpurun_out/r03_nb_tests.log 2>&1 || { tail -40 gpurun_out/r03_nb_tests.log; exit 1; }
tail -1 gpurun_out/r03_nb_tests.log
bash tools/ab.sh k128 3 build/nb3/libsgm_hip.so build/nb4/libsgm_hip.so build/nb2/libsgm_hip.so || exit 1
bash tools/ab.sh hd256 1 build/nb3/libsgm_hip.so build/nb4/libsgm_hip.so || exit 1
