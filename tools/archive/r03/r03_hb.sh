#!/bin/bash
# H pairs per backward band on a side stream (SGM_HPAIR_BANDS=1): parity, then paired timing.
set -o pipefail
mkdir -p gpurun_out
SGM_HPAIR_BANDS=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_fuzz.py tests/test_gpu_schedules.py "tests/test_gpu_fullsize.py::test_fullsize_vs_oracle[HD256_lr]" \
  "tests/test_gpu_fullsize.py::test_4k256_lr_vs_lean_oracle" > gpurun_out/r03_hb_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03_hb_tests.log; exit 1; }
tail -1 gpurun_out/r03_hb_tests.log
bash tools/ab_env.sh hd256 2 SGM_HPAIR_BANDS 0 1 || exit 1
bash tools/ab_env.sh 4k256 1 SGM_HPAIR_BANDS 0 1 || exit 1
