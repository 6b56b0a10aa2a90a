#!/bin/bash
# Census fused into cost_h (one view, D=128): parity, then paired timing (SGM_FUSED_CENSUS 0/1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_schedules.py tests/test_gpu_view_split.py \
  tests/test_gpu_gpu_sgm.py tests/test_cpp_surface.py "tests/test_gpu_fullsize.py::test_fullsize_vs_oracle" \
  > gpurun_out/r03_fct_tests.log 2>&1 || { tail -60 gpurun_out/r03_fct_tests.log; exit 1; }
tail -1 gpurun_out/r03_fct_tests.log
bash tools/ab_env.sh k128 4 SGM_FUSED_CENSUS 0 1 || exit 1
