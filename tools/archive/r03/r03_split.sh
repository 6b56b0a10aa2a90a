#!/bin/bash
# Split-row cost_h: parity (forced on, short warm-ups, full frames), then paired timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_costh_split.py tests/test_gpu_parity.py tests/test_gpu_real_texture.py \
  "tests/test_gpu_fullsize.py::test_fullsize_vs_oracle" > gpurun_out/r03_split_tests.log 2>&1 \
  || { tail -60 gpurun_out/r03_split_tests.log; exit 1; }
tail -1 gpurun_out/r03_split_tests.log
bash tools/ab_env.sh k128 3 SGM_COSTH_SPLIT 0 1 || exit 1
bash tools/ab_env.sh k128lr 2 SGM_COSTH_SPLIT 0 1 || exit 1
bash tools/ab_env.sh k64 2 SGM_COSTH_SPLIT 0 1 || exit 1
